"""Microbenchmark: id sort (hipCUB radix SortPairs) vs torch.sort at DeepFM batch sizes."""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import hipfm  # noqa: E402
from hipfm.ops import kernels as KN  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


def main():
    dev = torch.device("cuda", 0)
    for n in (39 * 1024, 39 * 16384, 39 * 32768, 39 * 65536):
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
            print(f"n={n:8d} bits={bits}: onesweep {t0:8.1f} us  lsd {tl:8.1f} us  hipcub SortPairs {t1:8.1f} us   "
                  f"torch.sort {t2:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
