"""Repeat the gather-fused tower launch on fixed inputs and report which outputs differ."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hipfm  # noqa: E402,F401
from hipfm.data.synthetic import make_synth  # noqa: E402
from hipfm.models.deepfm import NativeDeepFM  # noqa: E402
from hipfm.ops import kernels as KN  # noqa: E402


def main():
    preset = sys.argv[1] if len(sys.argv) > 1 else "total:6000"
    train = (sys.argv[2] if len(sys.argv) > 2 else "1") == "1"
    pad = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    dev = torch.device("cuda", 0)
    synth = make_synth(preset, seed=2024)
    B = 16384
    m = NativeDeepFM(synth.feature_size, synth.F, 8, [128, 64, 32], [0.5, 0.5, 0.5], l2_reg=1e-4,
                     learning_rate=5e-4, optimizer="Adam", sparse_update="lazy", seed=1234,
                     batch_size=B, device=dev, field_ranges=synth.field_ranges())
    ids, vals, lab = synth.batch(B, step=3, device=dev, id_dtype=torch.int32)
    if pad:
        base = m._tower_lds_layout

        def padded():
            h, d, x, x8, nb = base()
            return h, d, x, x8, nb + pad
        m._tower_lds_layout = padded
    m.stage_batch(ids, vals, lab)
    outs = []
    for rep in range(6):
        a = m._tower_args(B, train=train, gather=(m.idx, m.tv, m.tw))
        KN.tower(a, KE=m.K)
        torch.cuda.synchronize()
        o = {"prob": m.prob.clone(), "S": m.S.clone(), "y_fm": m.y_fm.clone()}
        if train:
            o.update(Et=m.Et.clone(), dX0=m.dX0.clone(), dlogit=m.dlogit.clone(),
                     **{f"Ht{i}": m.Ht[i].clone() for i in range(2)},
                     **{f"dZt{i}": m.dZt[i].clone() for i in range(3)})
        outs.append(o)
    for rep in range(1, 6):
        diff = {k: int((v != outs[0][k]).sum()) for k, v in outs[rep].items() if not torch.equal(v, outs[0][k])}
        print(f"rep {rep}: {diff if diff else 'equal'}")
        if "prob" in diff:
            bad = (outs[rep]["prob"] != outs[0]["prob"]).nonzero().reshape(-1)[:6].tolist()
            print("   prob rows", bad)
        for k in ("Et", "Ht0", "Ht1"):
            if k in diff:
                d = (outs[rep][k] != outs[0][k]).nonzero()[:6].tolist()
                print(f"   {k} [col,row] {d}")


if __name__ == "__main__":
    main()
