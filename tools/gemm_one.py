#!/usr/bin/env python
"""One wide-layer GEMM shape, one tile, repeated (profiling target for rocprofv3 passes):
  python tools/gemm_one.py --tile 9 --M 16384 --N 4096 --K 4096 --epi f32 --reps 20"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tile", type=int, default=9)
    ap.add_argument("--M", type=int, default=16384)
    ap.add_argument("--N", type=int, default=4096)
    ap.add_argument("--K", type=int, default=4096)
    ap.add_argument("--epi", default="f32", choices=["f32", "fwd", "torch"])
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    import hipfm  # noqa: F401
    from hipfm.ops import kernels as KN
    from hipfm.ops._lib import EpiArgs
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    A = (torch.rand(a.M, a.K, generator=g, device=dev) * 2 - 1).bfloat16()
    B = (torch.rand(a.N, a.K, generator=g, device=dev) * 2 - 1).bfloat16()
    if a.epi == "torch":
        for _ in range(a.reps):
            torch.matmul(A, B.t())
        torch.cuda.synchronize()
        return
    out = torch.zeros(a.M, a.N, device=dev)
    bias = torch.zeros(a.N, device=dev)
    step = torch.zeros(1, dtype=torch.int64, device=dev)
    ep = EpiArgs()
    ep.out, ep.bias, ep.step = out.data_ptr(), bias.data_ptr(), step.data_ptr()
    kind = KN.EPI_F32
    if a.epi == "fwd":
        o16 = torch.zeros(a.M, a.N, device=dev).bfloat16()
        ot = torch.zeros(a.N, a.M, device=dev).bfloat16()
        ep.out, ep.out_t, kind = o16.data_ptr(), ot.data_ptr(), KN.EPI_FWD
    for _ in range(a.reps):
        KN.gemm_nt(kind, a.tile, A, a.K, B, a.K, a.M, a.N, a.K, 1, ep)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
