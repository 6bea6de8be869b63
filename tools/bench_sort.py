"""Microbenchmark: id sorts at DeepFM batch sizes, timed as HIP-graph replays (the way the train
step runs them; eager timing would mostly measure host launch cost)."""
import os
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import hipfm  # noqa: E402
from hipfm.ops import kernels as KN  # noqa: E402


def timeit(fn, reps=20, inner=10):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g):
            for _ in range(inner):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / (reps * inner) * 1e6


def field_main(dev):
    """Per-field LDS sort (field_sort.hip) vs the global onesweep sort on Criteo-1TB-shape ids."""
    import math
    from hipfm.data.synthetic import make_synth
    synth = make_synth("criteo_1tb")
    F = synth.F
    for B in (1024, 4096, 8192, 16384):
        fs = KN.FieldSort(synth.field_ranges(), B, dev, max_pb=int(os.environ.get("HIPFM_FS_MAX_PB", "4")))
        n = B * F
        ids = synth.batch(B, 0, device=dev, id_dtype=torch.int32)[0].reshape(-1).contiguous()
        sk, perm = torch.empty_like(ids), torch.empty_like(ids)
        temp = torch.empty(KN.radix_temp_bytes(n) + 256, dtype=torch.uint8, device=dev)
        tf = timeit(lambda: fs(ids, B, sk, perm))
        t0 = timeit(lambda: KN.onesweep_sort_ids(ids, sk, perm, n, 30, temp))
        fs(ids, B, sk, perm)
        rk, rp = torch.sort(ids.long(), stable=True)
        ok = torch.equal(sk.long(), rk) and torch.equal(perm.long(), rp) and int(fs.err.item()) == 0
        print(f"criteo_1tb B={B:6d} n={n:8d}: field_sort {tf:7.1f} us  onesweep {t0:7.1f} us  exact={ok}",
              flush=True)


def run_main(dev):
    """Run-level sort (fsort_run.h) of G Criteo-1TB-shape batches vs G per-step field sorts."""
    from hipfm.data.synthetic import make_synth
    synth = make_synth("criteo_1tb")
    F, B = synth.F, 16384
    fs = KN.FieldSort(synth.field_ranges(), B, dev, max_pb=0)
    for G in (1, 4, 20):
        ids = [synth.batch(B, s, device=dev, id_dtype=torch.int32)[0].reshape(-1).contiguous() for s in range(G)]
        outs = [(torch.empty_like(i), torch.empty_like(i)) for i in ids]
        plan = fs.run_plan([(i, B, False, k, p) for i, (k, p) in zip(ids, outs)])
        tr = timeit(lambda: fs.run_sort(plan), reps=10, inner=5)
        ts = timeit(lambda: [fs(i, B, k, p) for i, (k, p) in zip(ids, outs)], reps=10, inner=5)
        print(f"criteo_1tb B={B} G={G:3d}: run_sort {tr:8.1f} us ({tr / G:6.1f}/batch)  "
              f"per-step field_sort x G {ts:8.1f} us", flush=True)


def main():
    dev = torch.device("cuda", 0)
    if "--field" in sys.argv:
        return field_main(dev)
    if "--run" in sys.argv:
        return run_main(dev)
    sizes = (39 * 1024, 39 * 16384, 39 * 32768, 39 * 65536)
    if "--only" in sys.argv:
        sizes = (int(sys.argv[sys.argv.index("--only") + 1]),)
    for n in sizes:
        for bits in (21, 30):
            keys = torch.randint(0, 1 << bits, (n,), dtype=torch.int32, device=dev)
            sk = torch.empty_like(keys)
            perm = torch.empty_like(keys)
            tmp = torch.empty_like(keys)
            temp = torch.empty(max(KN.sort_temp_bytes(n, bits), KN.radix_temp_bytes(n)) + 256,
                               dtype=torch.uint8, device=dev)
            t0 = timeit(lambda: KN.onesweep_sort_ids(keys, sk, perm, n, bits, temp))
            tl = timeit(lambda: KN.lsd_sort_ids(keys, sk, perm, n, bits, temp))
            t1 = timeit(lambda: KN.cub_sort_ids(keys, sk, tmp, perm, n, bits, temp))
            t2 = timeit(lambda: torch.sort(keys, stable=True))
            KN.onesweep_sort_ids(keys, sk, perm, n, bits, temp)
            ref_k, ref_p = torch.sort(keys.long(), stable=True)
            ok = torch.equal(sk.long(), ref_k) and torch.equal(perm.long(), ref_p)
            if not os.environ.get("HIPFM_OS_DEBUG_NOLB"):
                assert KN.sort_error(temp) == 0 and ok, "onesweep sort mismatch"
            print(f"n={n:8d} bits={bits}: onesweep {t0:8.1f} us  lsd {tl:8.1f} us  hipcub SortPairs {t1:8.1f} us   "
                  f"torch.sort {t2:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
