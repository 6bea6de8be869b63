#!/usr/bin/env python
"""Per-layer GEMM throughput at the reference's GPU tower (deep_layers 4096,4096,4096, B = 16384;
DOC p.37): the wide-layer LDS-staged tile (mlp.hip tile 8), the register-fed tile the model picked
before it, and torch.matmul (hipBLASLt) on the SAME bf16 operands, interleaved in one process
(rounds x variants, median and min reported).  Prints one JSON line per shape.

  python tools/gemm_bench.py [--batch 16384] [--width 4096] [--k0 320] [--rounds 5] [--reps 10]
"""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--width", type=int, default=4096)
    ap.add_argument("--k0", type=int, default=320)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--nodrop", action="store_true", help="forward epilogue without its dropout mask")
    args = ap.parse_args()
    import torch
    import hipfm  # noqa: F401
    from hipfm.models.deepfm import _pick_splitk, _pick_tile
    from hipfm.ops import kernels as KN
    from hipfm.ops._lib import EpiArgs

    dev = torch.device("cuda", 0)
    Bt, W = args.batch, args.width
    # (name, M, N, K, epilogue, split-K): NT GEMMs C[M,N] = A[M,K] . B[N,K]^T as the tower issues them
    shapes = [("fwd_layer0", Bt, W, args.k0, KN.EPI_FWD, 1),
              ("fwd_layer1", Bt, W, W, KN.EPI_FWD, 1),
              ("dgrad_layer1", Bt, W, W, KN.EPI_DGRAD, 1),
              ("wgrad_layer1", W, W, Bt, KN.EPI_F32, None)]
    g = torch.Generator(device=dev).manual_seed(0)
    for name, M, N, K, epi, split in shapes:
        A = (torch.rand(M, K, generator=g, device=dev) * 2 - 1).bfloat16()
        B = (torch.rand(N, K, generator=g, device=dev) * 2 - 1).bfloat16()
        bias = torch.zeros(N, device=dev)
        step = torch.zeros(1, dtype=torch.int64, device=dev)
        hprev = torch.ones(M, N, device=dev).bfloat16()
        old = _pick_tile(M, N, row_major_stream=(epi != KN.EPI_F32), allow_lds=False)
        variants = {}
        for tile in (13, 12, 11, 10, 9, KN.TILE_LDS, old):
            s = split if split is not None else _pick_splitk(M, N, K, tile)
            if tile in (KN.TILE_LDS, 9, 10, 11, 12, 13):
                while s > 1 and K % (64 * s):
                    s -= 1
            out = torch.zeros(s, M, N, device=dev) if epi == KN.EPI_F32 else torch.zeros(M, N, device=dev).bfloat16()
            out_t = torch.zeros(N, M, device=dev).bfloat16() if epi != KN.EPI_F32 else None
            ep = EpiArgs()
            ep.bias, ep.step, ep.out = bias.data_ptr(), step.data_ptr(), out.data_ptr()
            ep.out_t = out_t.data_ptr() if out_t is not None else 0
            ep.scale, ep.keep_thr, ep.drop = 2.0, 0x7FFFFFFF, 1 if (epi == KN.EPI_FWD and not args.nodrop) else 0
            if epi == KN.EPI_DGRAD:
                ep.hprev = hprev.data_ptr()
            variants[f"tile{tile}" + {8: "_lds", 9: "_pp", 10: "_pp3", 11: "_rb", 12: "_p8", 13: "_r8"}.get(tile, "_old")] = (
                lambda tile=tile, s=s, ep=ep: KN.gemm_nt(epi, tile, A, K, B, K, M, N, K, s, ep), (out, out_t, s))
        variants["torch_matmul"] = (lambda: torch.matmul(A, B.t()), None)
        times = {k: [] for k in variants}
        for fn, _ in variants.values():
            fn()
        torch.cuda.synchronize()
        for _ in range(args.rounds):
            for k, (fn, _) in variants.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1) / args.reps)
        flop = 2.0 * M * N * K
        res = {"shape": name, "M": M, "N": N, "K": K}
        for k, ts in times.items():
            res[k] = {"ms_median": round(statistics.median(ts), 4), "ms_min": round(min(ts), 4),
                      "tflops_median": round(flop / statistics.median(ts) / 1e9, 1)}
        res["lds_vs_torch"] = round(res["torch_matmul"]["ms_median"] / res["tile8_lds"]["ms_median"], 3)
        res["pp_vs_torch"] = round(res["torch_matmul"]["ms_median"] / res["tile9_pp"]["ms_median"], 3)
        res["pp3_vs_torch"] = round(res["torch_matmul"]["ms_median"] / res["tile10_pp3"]["ms_median"], 3)
        res["rb_vs_torch"] = round(res["torch_matmul"]["ms_median"] / res["tile11_rb"]["ms_median"], 3)
        res["r8_vs_torch"] = round(res["torch_matmul"]["ms_median"] / res["tile13_r8"]["ms_median"], 3)
        res["p8_vs_torch"] = round(res["torch_matmul"]["ms_median"] / res["tile12_p8"]["ms_median"], 3)
        # numerics spot check of the LDS tile against torch (fp32-accumulated products of bf16)
        if epi == KN.EPI_F32:
            _, (out, _, s) = variants["tile13_r8"]
            variants["tile13_r8"][0]()
            torch.cuda.synchronize()
            ref = torch.matmul(A.float(), B.float().t())
            res["max_rel_err"] = float((out.sum(0) - ref).abs().max() / ref.abs().max())
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
