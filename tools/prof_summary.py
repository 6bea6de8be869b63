"""Summarise a rocprofv3 --kernel-trace --stats run into markdown (for profiles/).

usage: python tools/prof_summary.py <prof_dir> <out.md> [title]
Writes the top kernels by total time and one steady-state training step's kernel timeline
(one period between two consecutive dense-optimizer kernels: dense_opt, or finalize_opt when
the optimizer rides on the gradient finalize; formerly step_inc).
"""
import csv
import glob
import os
import sys


def main():
    d, out = sys.argv[1], sys.argv[2]
    title = sys.argv[3] if len(sys.argv) > 3 else os.path.basename(d.rstrip("/"))
    stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    trace = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    lines = [f"# {title}", ""]
    bench = os.path.join(d, "bench.log")
    if os.path.exists(bench):
        js = [l for l in open(bench) if l.startswith("{")]
        if js:
            lines += ["bench line (under the profiler):", "", "```", js[-1].strip(), "```", ""]
    if stats:
        rows = list(csv.DictReader(open(stats[0])))
        rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
        lines += ["## Top kernels (whole run, incl. warm-up / data generation / eval)", "",
                  "| total us | calls | avg us | % | kernel |", "|---:|---:|---:|---:|---|"]
        for r in rows[:25]:
            lines.append(f"| {float(r['TotalDurationNs'])/1e3:.1f} | {r['Calls']} | "
                         f"{float(r['AverageNs'])/1e3:.2f} | {float(r['Percentage']):.1f} | "
                         f"`{r['Name'][:90]}` |")
        lines.append("")
    if trace:
        rows = list(csv.DictReader(open(trace[0])))
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        # one step = from the end of one step-closing kernel (the one that advances the step
        # counter: dense optimizer / fused finalize / wgfin / sparse+wgfin) to the end of the next;
        # the median-span step of the timed steps (graph replays) is listed
        idx = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(
            ("step_inc", "void dense_opt_kernel", "void finalize_opt_kernel", "void wgfin_kernel<0",
             "void sfwg_kernel", "void sh_apply_dense_kernel"))]
        pairs = [(a, b, int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"]))
                 for a, b in zip(idx, idx[1:])]
        pairs = [p for p in pairs if p[2] < 1_000_000]       # steps, not eval / setup gaps
        if pairs:
            spans = sorted(p[2] for p in pairs)
            med = spans[len(spans) // 2]
            a, b, _ = min(pairs, key=lambda p: abs(p[2] - med))
            t0 = int(rows[a]["End_Timestamp"])
            lines += ["## One steady-state training step (graph replay; the median-span step)", "",
                      f"{len(spans)} consecutive step spans: min {spans[0]/1e3:.1f} us, median "
                      f"{med/1e3:.1f} us, max {spans[-1]/1e3:.1f} us", "",
                      "| start us | dur us | kernel |", "|---:|---:|---|"]
            tot = 0
            for r in rows[a + 1: b + 1]:
                s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                tot += e - s
                lines.append(f"| {(s - t0)/1e3:.2f} | {(e - s)/1e3:.2f} | `{r['Kernel_Name'][:80]}` |")
            span = (int(rows[b]["End_Timestamp"]) - t0) / 1e3
            lines += ["", f"step span {span:.1f} us, sum of kernel durations {tot/1e3:.1f} us", ""]
        # run-level sort / routing (multi-step graphs): the kernels from a run's sort to its
        # first tower, for the median-length run start
        starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("fs2_sort_run_kernel")]
        spans = []
        for i in starts:
            j = next((k for k in range(i + 1, len(rows)) if rows[k]["Kernel_Name"].startswith("void tower_kernel")),
                     None)
            if j is not None:
                spans.append((int(rows[j]["Start_Timestamp"]) - int(rows[i]["Start_Timestamp"]), i, j))
        if spans:
            spans.sort()
            d, i, j = spans[len(spans) // 2]
            t0 = int(rows[i]["Start_Timestamp"])
            lines += ["## Run start (run-level sort / routing, median of %d runs): %.1f us to the first tower"
                      % (len(spans), d / 1e3), "", "| start us | dur us | kernel |", "|---:|---:|---|"]
            for r in rows[i:j]:
                s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                lines.append(f"| {(s - t0)/1e3:.2f} | {(e - s)/1e3:.2f} | `{r['Kernel_Name'][:80]}` |")
            lines.append("")
        # every multi-step graph replay in order (the bench's timed window is the last long one
        # before eval): steps, run span from the sort's start, sort time and median step span
        if starts:
            closers = set(idx) if trace else set()
            lines += ["## Every run (graph replay) in order", "",
                      "| run | steps | span us | sort+routing us | median step us | max step us |",
                      "|---:|---:|---:|---:|---:|---:|"]
            for n_, i in enumerate(starts):
                hi = starts[n_ + 1] if n_ + 1 < len(starts) else len(rows)
                ends, last = [], int(rows[i]["End_Timestamp"])
                for k in range(i + 1, hi):
                    if int(rows[k]["Start_Timestamp"]) - last > 1_000_000:
                        break                      # an idle gap: the run has ended
                    last = max(last, int(rows[k]["End_Timestamp"]))
                    if k in closers:
                        ends.append(int(rows[k]["End_Timestamp"]))
                if not ends:
                    continue
                j = next((k for k in range(i + 1, hi) if rows[k]["Kernel_Name"].startswith("void tower_kernel")), i)
                st = [b - a for a, b in zip(ends, ends[1:])]
                st.sort()
                lines.append(f"| {n_} | {len(ends)} | {(ends[-1] - int(rows[i]['Start_Timestamp'])) / 1e3:.1f} | "
                             f"{(int(rows[j]['Start_Timestamp']) - int(rows[i]['Start_Timestamp'])) / 1e3:.1f} | "
                             f"{(st[len(st) // 2] / 1e3) if st else 0:.1f} | {(st[-1] / 1e3) if st else 0:.1f} |")
            lines.append("")
    open(out, "w").write("\n".join(lines) + "\n")
    print(out)


if __name__ == "__main__":
    main()
