#!/usr/bin/env python
"""GPU Example decode throughput (csrc/kernels/decode.hip) on one batch of Kaggle-shape records
(F = 39), with and without the device-side data CRC: median ms per batch over repeats.

  python tools/decode_bench.py [--rows 16384] [--reps 50]"""
import argparse
import json
import os
import statistics
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=16384)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    import numpy as np
    import torch
    import hipfm  # noqa: F401
    from hipfm.data import tfrecord as tr
    from hipfm.ops import kernels as KN
    F, B = 39, a.rows
    rng = np.random.default_rng(0)
    ids = rng.integers(0, 1 << 20, size=(B, F))
    vals = rng.random((B, F), dtype=np.float32)
    lab = (rng.random(B) < 0.3).astype(np.float32)
    recs = [tr.encode_example(float(lab[i]), [int(x) for x in ids[i]], [float(v) for v in vals[i]]) for i in range(B)]
    dev = torch.device("cuda", 0)
    out = {"rows": B, "bytes_per_record": sum(map(len, recs)) / B}
    for crc in (False, True):
        blob = b"".join(r + (struct.pack("<I", tr.masked_crc32c(r)) if crc else b"") for r in recs)
        offs = np.zeros(B + 1, dtype=np.int64)
        offs[1:] = np.cumsum([len(r) + (4 if crc else 0) for r in recs])
        draw = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
        doffs = torch.from_numpy(offs.astype(np.int32)).to(dev)
        i_ = torch.empty(B, F, dtype=torch.int32, device=dev)
        v_ = torch.empty(B, F, device=dev)
        l_ = torch.empty(B, device=dev)
        err = torch.tensor([0, 0x7FFFFFFF], dtype=torch.int32, device=dev)
        ts = []
        for r in range(a.reps + 5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            KN.decode_examples(draw, doffs, B, F, 0, i_, v_, l_, err, crc=crc)
            e1.record()
            torch.cuda.synchronize()
            if r >= 5:
                ts.append(e0.elapsed_time(e1))
        assert err.tolist() == [0, 0x7FFFFFFF], err.tolist()
        assert torch.equal(i_.cpu(), torch.from_numpy(ids.astype(np.int32)))
        out["ms_crc" if crc else "ms"] = round(statistics.median(ts), 4)
    out["Mrows_per_s"] = round(B / out["ms"] / 1e3, 1)
    out["Mrows_per_s_crc"] = round(B / out["ms_crc"] / 1e3, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
