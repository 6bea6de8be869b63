"""Which rows differ between the tf1_dense split form and the scatter + sweep form after eager
steps (tests/test_gpu_tf1.py): batch rows or swept rows, and by how much."""
import sys

import torch

import hipfm  # noqa: F401
import hipfm.models.deepfm as dm
from hipfm.data.synthetic import make_synth
from hipfm.models.deepfm import NativeDeepFM

DEV = torch.device("cuda", 0)


def main(mode="merged", opt="Adam", K=8, steps=1, nxt=0):
    dm._SWEEP_MODE = mode
    synth = make_synth("criteo_kaggle")
    B = 2048
    kw = dict(optimizer=opt, sparse_update="tf1_dense", batch_size=B, device=DEV, seed=7,
              field_ranges=synth.field_ranges(), l2_reg=1e-3, adam_epsilon=1e-2)
    dm._TF1_SPLIT = True
    a = NativeDeepFM(synth.feature_size, synth.F, K, [64, 32], [0.5, 0.5], **kw)
    dm._TF1_SPLIT = False
    b = NativeDeepFM(synth.feature_size, synth.F, K, [64, 32], [0.5, 0.5], **kw)
    pool = [synth.batch(B, i, device=DEV, id_dtype=torch.int32) for i in range(steps + 1)]
    seen = torch.zeros(a.R, dtype=torch.bool, device=DEV)
    for i in range(steps):
        n = pool[i + 1][0] if nxt else None
        a.train_step(*pool[i], next_ids=n)
        b.train_step(*pool[i], next_ids=n)
        seen[pool[i][0].reshape(-1).long()] = True
        torch.cuda.synchronize()
        dv = (a.tv != b.tv).any(dim=1) | (a.tw != b.tw)
        for s, t in zip(a.sv, b.sv):
            dv |= (s != t).reshape(a.R, -1).any(dim=1)
        cur = torch.zeros_like(seen)
        cur[pool[i][0].reshape(-1).long()] = True
        print(f"step {i}: rows differing {int(dv.sum())} (in this batch {int((dv & cur).sum())}, "
              f"outside {int((dv & ~cur).sum())}); batch rows {int(cur.sum())}; "
              f"max |dtv| {(a.tv - b.tv).abs().max().item():.3e}; dense equal {torch.equal(a.p, b.p)}",
              flush=True)
        if int(dv.sum()):
            r = torch.nonzero(dv).flatten()[:5]
            for x in r.tolist():
                print("  row", x, "in batch", bool(cur[x]), "a", a.tv[x].tolist()[:3], "b", b.tv[x].tolist()[:3])


if __name__ == "__main__":
    args = sys.argv[1:]
    main(args[0] if args else "merged", args[1] if len(args) > 1 else "Adam", int(args[2]) if len(args) > 2 else 8,
         int(args[3]) if len(args) > 3 else 2, int(args[4]) if len(args) > 4 else 0)
