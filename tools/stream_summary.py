"""Summarise a rocprofv3 --kernel-trace --memory-copy-trace run of the streamed input path
(scripts/stream_prof.sh): the host-to-device copies (count, bytes, bandwidth) and, over the
last streamed epoch's window, how much of the wall time the GPU spent in kernels, in copies,
and in neither.

usage: python tools/stream_summary.py <prof_dir>
"""
import csv
import glob
import os
import sys


def _rows(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def _union(iv):
    """Total length of a union of [s, e) intervals."""
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    d = sys.argv[1]
    ks = _rows(d, "*kernel_trace.csv")
    cs = _rows(d, "*memory_copy_trace.csv")
    print("# streamed input path: copies and kernels\n")
    if cs:
        print("memory-copy columns:", ", ".join(cs[0].keys()), "\n")
    bycol = None
    for c in ("Bytes", "Size", "Copy_Bytes", "Num_Bytes"):
        if cs and c in cs[0]:
            bycol = c
    dirs = {}
    for r in cs:
        k = r.get("Direction", r.get("Kind", "?"))
        n = int(r[bycol]) if bycol else 0
        t = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        a = dirs.setdefault(k, [0, 0, 0])
        a[0] += 1
        a[1] += n
        a[2] += t
    print("| direction | copies | MB | busy ms | GB/s while copying |\n|---|---:|---:|---:|---:|")
    for k, (n, b, t) in sorted(dirs.items()):
        print(f"| {k} | {n} | {b / 1e6:.1f} | {t / 1e6:.2f} | {b / max(t, 1):.1f} |")
    if not ks:
        return
    # the streamed-epoch window: the last third of the training kernels' span (epoch 2 of 3)
    tk = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in ks]
    tr = [x for x in tk if x[2].startswith(("void tower", "void sfwg", "fs2_sort_run"))]
    if not tr:
        return
    t0, t1 = tr[0][0], tr[-1][1]
    w0 = t0 + 2 * (t1 - t0) // 3
    kin = [(max(s, w0), e) for s, e, _ in tk if e > w0 and s < t1]
    cin = [(max(int(r["Start_Timestamp"]), w0), int(r["End_Timestamp"])) for r in cs
           if int(r["End_Timestamp"]) > w0 and int(r["Start_Timestamp"]) < t1]
    h2d = [(max(int(r["Start_Timestamp"]), w0), int(r["End_Timestamp"])) for r in cs
           if int(r["End_Timestamp"]) > w0 and int(r["Start_Timestamp"]) < t1 and
           "HOST_TO_DEVICE" in r.get("Direction", "").upper()]
    wall = t1 - w0
    kb, cb, hb = _union(kin), _union(cin), _union(h2d)
    both = kb + cb - _union(kin + cin)
    steps = sum(1 for s, e, n in tk if s >= w0 and n.startswith("void tower"))
    print(f"\nlast-third window: {wall / 1e6:.2f} ms, {steps} training steps "
          f"({wall / 1e3 / max(steps, 1):.1f} us per step)")
    print(f"- kernels busy {kb / 1e6:.2f} ms ({100 * kb / wall:.0f} %), copies busy {cb / 1e6:.2f} ms "
          f"({100 * cb / wall:.0f} %; host-to-device {100 * hb / wall:.0f} %), both at once "
          f"{both / 1e6:.2f} ms, GPU idle {(wall - _union(kin + cin)) / 1e6:.2f} ms")
    names = {}
    for s, e, n in tk:
        if s >= w0:
            a = names.setdefault(n.split("(")[0][:60], [0, 0])
            a[0] += 1
            a[1] += e - s
    print("\n| kernel (window) | calls | us total | us per step |\n|---|---:|---:|---:|")
    for n, (c, t) in sorted(names.items(), key=lambda x: -x[1][1])[:15]:
        print(f"| `{n}` | {c} | {t / 1e3:.0f} | {t / 1e3 / max(steps, 1):.1f} |")


if __name__ == "__main__":
    main()
