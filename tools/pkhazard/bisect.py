"""Packed-FP32 hazard bisection (tools/pkhazard/README.md): the gather-fused tower's eval launch
repeated on identical inputs with the kernel library named by HIPFM_KERNELS_SO (a packed build,
optionally stopped after a phase: -DTW_BISECT=1 after the gather, 2 after the forward layers);
counts launches whose FM logits differ from the first launch and from a float64 host reference.
usage: HIPFM_KERNELS_SO=... python tools/pkhazard/bisect.py [launches]"""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
import hipfm  # noqa: E402,F401
from hipfm.data.synthetic import make_synth  # noqa: E402
from hipfm.models.deepfm import NativeDeepFM  # noqa: E402
from hipfm.ops import kernels as KN  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    B = 16384
    synth = make_synth("criteo_kaggle", seed=2024)
    m = NativeDeepFM(synth.feature_size, synth.F, 8, [128, 64, 32], [1.0, 1.0, 1.0], batch_size=B,
                     device="cuda", field_ranges=synth.field_ranges(), sparse_update="lazy")
    ids, vals, _ = synth.batch(B, step=500_000, device="cuda", id_dtype=torch.int32)
    m.stage_batch(ids, vals, None)
    a = m._tower_args(B, train=False, with_labels=False, gather=m._fm_inputs(B, train=False))
    idl = ids.long()
    v = m.tv[idl].double() * vals.double().unsqueeze(-1)
    w = m.tw[idl].double() * vals.double()
    fb = float(m.p[m.dense_segs["fm_bias"].off])
    ex = fb + w.sum(1) + 0.5 * (v.sum(1) ** 2 - (v * v).sum(1)).sum(1)
    first, diff_first, bad_ref, worst, rows = None, 0, 0, 0.0, 0
    for _ in range(n):
        m.y_fm.zero_()
        KN.tower(a, KE=m.K)
        torch.cuda.synchronize()
        y = m.y_fm[:B].clone()
        if first is None:
            first = y
        elif not torch.equal(y, first):
            diff_first += 1
            rows += int((y != first).sum())
        e = float((y.double() - ex).abs().max())
        worst = max(worst, e)
        bad_ref += e > 1e-6
    print(f"{os.path.basename(os.environ.get('HIPFM_KERNELS_SO', 'default'))}: {n} launches, "
          f"{diff_first} differ from the first ({rows} rows), {bad_ref} off the float64 reference "
          f"(worst {worst:.3e})", flush=True)


if __name__ == "__main__":
    main()
