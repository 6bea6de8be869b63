"""Phase-stamp analysis of the diagnostic stamp build (HIPFM_BUILD_STAMPS=1, csrc/kernels/common.h
HFM_STAMP): per workgroup, 100-MHz wall-clock stamps at the phase boundaries of the tower and of
the sparse + wgfin launch (last timed step of a bench run).

usage:
  HIPFM_BUILD_STAMPS=1 python -m hipfm.ops.build                      # (on the CPU, in-tree)
  HIPFM_KERNELS_SO=<repo>/.../_lib/libhipfm_kernels_stamps.so HIPFM_BENCH_STAMPS=out.npz \
      python bench.py --steps 20 --warmup 5
  python tools/stamps.py out.npz [report.md]

For each buffer, workgroups are grouped by the set of stamps they wrote (e.g. sparse tiles vs
wgfin workgroups); per group: the spread of start times (dispatch), and per phase (consecutive
stamps) the p10 / median / p90 duration in microseconds; plus the launch span.
"""
import sys

import numpy as np

PHASES = {
    "hfm_st_tower": {0: "start", 1: "gather", 2: "E^T store", 3: "fwd L0", 4: "fwd L1", 5: "fwd L2",
                     7: "head+partials", 8: "dZ^T(L) store", 9: "dgrad L2->L1", 10: "dZ^T store",
                     11: "dgrad L1->L0", 12: "dZ^T store", 15: "dX0"},
    "hfm_st_sf": {0: "start", 1: "slot grads", 2: "heads", 3: "chunk sums", 4: "row updates",
                  5: "publish", 6: "look-back", 7: "arrive", 8: "wgfin start", 9: "wgfin"},
}


def analyze(path):
    d = np.load(path)
    lines = []
    for name in d.files:
        st = d[name].astype(np.int64)
        used = st[:, 0] != 0
        used |= st[:, 8] != 0
        idx = np.nonzero(used)[0]
        if len(idx) == 0:
            continue
        st = st[idx]
        t0 = st[st > 0].min()
        lines.append(f"## {name}: {len(idx)} workgroups, launch span "
                     f"{(st.max() - t0) / 100:.1f} us")
        groups = {}
        for r, row in zip(idx, st):
            key = tuple(int(k) for k in np.nonzero(row)[0])
            groups.setdefault(key, []).append((r, row))
        names = PHASES.get(name, {})
        for key, rows in sorted(groups.items(), key=lambda kv: -len(kv[1])):
            if len(rows) < 2:
                continue
            arr = np.array([row for _, row in rows])
            first = arr[:, key[0]]
            last = arr[:, key[-1]]
            lines.append("")
            lines.append(f"### {len(rows)} workgroups with stamps {list(key)} (blocks {rows[0][0]}..{rows[-1][0]})")
            lines.append(f"start offset us: p0 {(first.min() - t0) / 100:.1f}  p50 "
                         f"{(np.median(first) - t0) / 100:.1f}  p100 {(first.max() - t0) / 100:.1f}; "
                         f"end offset us: p50 {(np.median(last) - t0) / 100:.1f}  p100 {(last.max() - t0) / 100:.1f}; "
                         f"lifetime us: p50 {np.median(last - first) / 100:.2f}  p90 "
                         f"{np.percentile(last - first, 90) / 100:.2f}")
            lines.append("")
            lines.append("| phase | p10 us | median us | p90 us | max us |")
            lines.append("|---|---:|---:|---:|---:|")
            for a, b in zip(key[:-1], key[1:]):
                dt = (arr[:, b] - arr[:, a]) / 100.0
                lines.append(f"| {names.get(a, a)} -> {names.get(b, b)} | {np.percentile(dt, 10):.2f} | "
                             f"{np.median(dt):.2f} | {np.percentile(dt, 90):.2f} | {dt.max():.2f} |")
        lines.append("")
    return "\n".join(lines)


def main():
    txt = analyze(sys.argv[1])
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            f.write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
