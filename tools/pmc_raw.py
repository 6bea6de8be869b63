"""Raw per-kernel counter table of rocprofv3 --pmc runs: the mean of EVERY collected counter per
dispatch, one column per counter, plus derived occupancy / stall shares when the SQ wave counters
are present.

usage: python tools/pmc_raw.py <out.md> <title> <pmc_dir> [<pmc_dir> ...]

Derived (SQ_* wave counters count quad-cycles; MI355X_MICROARCH.md "rocprofv3 PMC slots"):
  waves/SIMD   SQ_WAVE_CYCLES / (SQ_BUSY_CYCLES x 4 SIMDs per CU ... ) is not exposed directly;
               we report mean resident waves per CU = SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / 8 x 256 / 4)
  wait %       SQ_WAIT_ANY / SQ_WAVE_CYCLES        (parked on s_waitcnt / barrier)
  issue-stall% SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES   (ready but not issued)
  active %     SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
"""
import collections
import csv
import glob
import os
import sys

from pmc_summary import OURS


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    if not f:
        return per, dur
    for r in csv.DictReader(open(f[0])):
        name = r["Kernel_Name"]
        if not any(k in name for k in OURS):
            continue
        key = name.split("(")[0][:48]
        per[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[key][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return per, dur


def main():
    out, title, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    ctr = collections.defaultdict(dict)
    durs = collections.defaultdict(list)
    names = []
    for d in dirs:
        per, dur = load(d)
        for k, cs in per.items():
            for c, v in cs.items():
                ctr[k][c] = sum(v) / len(v)
                if c not in names:
                    names.append(c)
            durs[k] += list(dur[k].values())
    hdr = ["kernel", "calls", "us"] + names
    derived = all(n in names for n in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"))
    if derived:
        hdr += ["wait %", "issue-stall %", "active %"]
    if "SQ_WAVE_CYCLES" in names and "GRBM_GUI_ACTIVE" in names:
        hdr += ["waves/CU"]
    lines = [f"# {title}", "", "Mean per dispatch. Sources: " +
             ", ".join(f"`{os.path.basename(d.rstrip('/'))}`" for d in dirs), "",
             "| " + " | ".join(hdr) + " |", "|" + "---|" * len(hdr)]
    for k in sorted(ctr, key=lambda k: -sum(durs[k])):
        c = ctr[k]
        n = len(durs[k]) // max(1, len(dirs))
        us = 1e6 * sum(durs[k]) / max(1, len(durs[k]))
        row = [f"`{k}`", str(n), f"{us:.1f}"] + [f"{c.get(x, float('nan')):.4g}" for x in names]
        if derived:
            w = max(1.0, c["SQ_WAVE_CYCLES"])
            row += [f"{100 * c['SQ_WAIT_ANY'] / w:.1f}", f"{100 * c['SQ_WAIT_INST_ANY'] / w:.1f}",
                    f"{100 * c['SQ_ACTIVE_INST_ANY'] / w:.1f}"]
        if "SQ_WAVE_CYCLES" in names and "GRBM_GUI_ACTIVE" in names:
            # GRBM_GUI_ACTIVE: summed over 8 XCDs (cycles); SQ_WAVE_CYCLES in quad-cycles, summed over CUs
            cyc = max(1.0, c["GRBM_GUI_ACTIVE"] / 8)
            row += [f"{4 * c['SQ_WAVE_CYCLES'] / (cyc * 256):.2f}"]
        lines.append("| " + " | ".join(row) + " |")
    with open(out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
