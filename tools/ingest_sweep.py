"""Host ingest rate of the native loader (csrc/io/hfm_io.cpp through data/native_io.py) over a
directory of TFRecords, for several decode-thread / copy-thread counts.
usage: python tools/ingest_sweep.py <dir> [F] [B]"""
import glob
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import hipfm  # noqa: E402,F401
from hipfm.data.native_io import NativeLoader  # noqa: E402


def rate(files, F, B, th, ct, n32=True, qd=4):
    lab = np.empty(B, np.float32)
    ids = np.empty((B, F), np.int32)
    vals = np.empty((B, F), np.float32)
    ld = NativeLoader(files, F, B, threads=th, copy_threads=ct, ids32=n32, queue_depth=qd)
    rows, t0 = 0, time.perf_counter()
    while True:
        r = ld.next_into(lab, ids, vals)
        if r == 0:
            break
        rows += r
    dt = time.perf_counter() - t0
    ld.close()
    return rows / dt


def main():
    d = sys.argv[1]
    F = int(sys.argv[2]) if len(sys.argv) > 2 else 39
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 16384
    files = sorted(glob.glob(f"{d}/tr*"))
    for rep in range(2):
        for th, ct, qd in ((16, 8, 4), (16, 8, 16), (16, 8, 64), (16, 4, 16), (12, 4, 16), (24, 8, 16)):
            print(f"threads {th:2d} copy {ct} queue depth {qd:2d}: {rate(files, F, B, th, ct, True, qd) / 1e6:.1f} M rows/s",
                  flush=True)


if __name__ == "__main__":
    main()
