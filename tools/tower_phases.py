"""Phase timing of the fused tower kernel (csrc/kernels/tower.hip TW_STAMP): per-workgroup
wall-clock stamps (100 MHz s_memrealtime) at the end of every forward layer, the head and every
dgrad step.  Prints median phase durations over workgroups and the spread of workgroup starts.

usage: python tools/tower_phases.py [B] [preset]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hipfm  # noqa: E402
from hipfm.data.synthetic import make_synth  # noqa: E402
from hipfm.models.deepfm import NativeDeepFM  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    synth = make_synth(sys.argv[2] if len(sys.argv) > 2 else "criteo_kaggle", seed=1)
    dev = torch.device("cuda", 0)
    m = NativeDeepFM(synth.feature_size, synth.F, 8, [128, 64, 32], [0.5] * 3, batch_size=B, device=dev,
                     sparse_update="lazy", field_ranges=synth.field_ranges())
    batches = [synth.batch(B, step=i, device=dev, id_dtype=torch.int32) for i in range(3)]
    for ids, vals, lab in batches:
        m.train_step(ids, vals, lab)
    torch.cuda.synchronize()
    grid = m.M // 32
    ts = torch.zeros(grid, 16, dtype=torch.int64, device=dev)
    orig = m._tower_args

    def stamped(*a, **k):
        t = orig(*a, **k)
        t.tstamp = ts.data_ptr()
        return t
    m._tower_args = stamped
    for rep in range(3):
        ids, vals, lab = batches[rep]
        m.train_step(ids, vals, lab)
        torch.cuda.synchronize()
    t = ts.cpu().double() * 10.0 / 1000.0          # 100 MHz ticks -> us
    nl = len(m.layers)
    names = [f"fwd layer {i}" for i in range(nl)] + ["head"] + [f"dgrad {nl - 1 - j}->{nl - 2 - j}"
                                                                for j in range(nl - 1)] + ["dX0"]
    cols = list(range(1, nl + 1)) + [9] + [10 + j for j in range(nl - 1)] + [15]
    prev = t[:, 0]
    print(f"B={B} workgroups={grid}  start spread {float(t[:, 0].max() - t[:, 0].min()):.2f} us, "
          f"kernel span {float(t[:, 15].max() - t[:, 0].min()):.2f} us, "
          f"median WG lifetime {float((t[:, 15] - t[:, 0]).median()):.2f} us")
    for n, c in zip(names, cols):
        d = t[:, c] - prev
        print(f"  {n:14s} median {float(d.median()):6.2f} us   p90 {float(d.quantile(0.9)):6.2f} us")
        prev = t[:, c]


if __name__ == "__main__":
    main()
