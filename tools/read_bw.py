#!/usr/bin/env python
"""Host file-read bandwidth of a dataset directory (the ceiling of any streamed-input design that
reads every record's bytes each epoch): N threads each read whole files with readinto into a
reused buffer (the GIL is released during the read), passes over the same files.

  python tools/read_bw.py <dir> [--threads 1,4,16] [--passes 2]"""
import argparse
import glob
import json
import os
import threading
import time


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--threads", default="1,4,16")
    ap.add_argument("--passes", type=int, default=2)
    a = ap.parse_args()
    files = sorted(f for f in glob.glob(os.path.join(a.dir, "**", "*"), recursive=True) if os.path.isfile(f))
    total = sum(os.path.getsize(f) for f in files)
    out = {"files": len(files), "bytes": total}
    for nt in [int(x) for x in a.threads.split(",")]:
        rates = []
        for _ in range(a.passes):
            todo = list(files)
            lock = threading.Lock()

            def work():
                buf = bytearray(64 << 20)
                mv = memoryview(buf)
                while True:
                    with lock:
                        if not todo:
                            return
                        f = todo.pop()
                    with open(f, "rb", buffering=0) as fh:
                        while fh.readinto(mv):
                            pass
            ts = [threading.Thread(target=work) for _ in range(nt)]
            t0 = time.perf_counter()
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            rates.append(round(total / (time.perf_counter() - t0) / 1e9, 2))
        out[f"GBps_threads{nt}"] = rates
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
