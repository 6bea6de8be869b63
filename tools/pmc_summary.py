"""Per-kernel PMC summary of rocprofv3 --pmc runs (scripts/pmc.sh) for profiles/.

usage: python tools/pmc_summary.py <out.md> <title> <pmc_dir> [<pmc_dir> ...]

For every hipfm kernel: mean duration per dispatch and the mean of each collected counter per
dispatch, plus derived rates: L2->CU fetch / write bandwidth (FETCH_SIZE / WRITE_SIZE are KB),
MFMA utilisation (SQ_VALU_MFMA_BUSY_CYCLES over SIMD-cycles of the kernel: 1024 SIMDs x 2.4 GHz),
MFMA TFLOP/s (MOPS x 512 per MFMA op) and LDS bank-conflict cycles per LDS instruction.
"""
import collections
import csv
import glob
import os
import sys

OURS = ("decode_examples", "head_wide", "shadow_transpose", "tower_kernel", "tower_light", "wgfin_kernel", "sfwg_kernel", "sfwg_x", "fs2_",  "dense_sweep", "fm_fwd", "wgrad_group", "finalize_kernel", "sf_tile", "sf_carry",
        "fs_sort", "fs_transpose", "dense_opt", "w8_quant", "sh_", "seg_", "onesweep", "lsd_",
        "gemm_nt", "gemm_lds", "gemm_pp", "Cijk", "head_kernel", "rcclGenericKernel")
SIMDS = 1024
HBM_BPS = 8e12       # MI355X HBM3E peak
BF16_PEAK_TF = 2500.0  # dense bf16 MFMA peak (no sparsity)
CLOCK_HZ = 2.4e9     # MI355X peak engine clock: MFMA util = busy SIMD-cycles / (SIMDs x duration x clock)


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return {}
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
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
    for d in dirs:
        got = load(d)
        if not got:
            continue
        per, dur = got
        for k, cs in per.items():
            for c, v in cs.items():
                ctr[k][c] = sum(v) / len(v)
            durs[k] += list(dur[k].values())
    lines = [f"# {title}", "", "Mean per dispatch over the profiled run (warm-up, timed steps, eval).",
             "Sources: " + ", ".join(f"`{os.path.basename(d.rstrip('/'))}`" for d in dirs), "",
             "| kernel | calls | us | fetch MB | fetch GB/s | write MB | write GB/s | HBM r+w % of 8 TB/s | "
             "MFMA util % | MFMA TF/s | % of 2.5 PF bf16 | LDS conflict cyc / LDS inst |",
             "|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|"]
    for k in sorted(ctr, key=lambda k: -sum(durs[k])):
        c = ctr[k]
        t = sum(durs[k]) / max(1, len(durs[k]))
        f = c.get("FETCH_SIZE")
        w = c.get("WRITE_SIZE")
        busy, gui = c.get("SQ_VALU_MFMA_BUSY_CYCLES"), c.get("GRBM_GUI_ACTIVE")
        mops = (c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) + c.get("SQ_INSTS_VALU_MFMA_MOPS_F8", 0.0))
        lds, conf = c.get("SQ_INSTS_LDS"), c.get("SQ_LDS_BANK_CONFLICT")

        def fmt(x, p=1):
            return "—" if x is None else f"{x:.{p}f}"
        util = None if busy is None else 100.0 * busy / (SIMDS * t * CLOCK_HZ)
        tf = None if not ("SQ_INSTS_VALU_MFMA_MOPS_BF16" in c or "SQ_INSTS_VALU_MFMA_MOPS_F8" in c) \
            else mops * 512 / t / 1e12
        hbm = None if f is None or w is None else 100.0 * (f + w) * 1024 / t / HBM_BPS
        lines.append(
            f"| `{k}` | {len(durs[k])} | {t * 1e6:.1f} | {fmt(None if f is None else f / 1024, 2)} | "
            f"{fmt(None if f is None else f * 1024 / t / 1e9, 0)} | {fmt(None if w is None else w / 1024, 2)} | "
            f"{fmt(None if w is None else w * 1024 / t / 1e9, 0)} | {fmt(hbm)} | {fmt(util)} | {fmt(tf, 2)} | "
            f"{fmt(None if tf is None else 100.0 * tf / BF16_PEAK_TF, 2)} | "
            f"{fmt(None if not lds else conf / lds, 3)} |")
    lines += ["", "MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x kernel duration x 2.4 GHz). "
              "The deep tower is 128/64/32 wide: its GEMMs are latency- and LDS-bound, not MFMA-bound; "
              "the embedding kernels (fm_fwd2, sf_tile) are gather/scatter bandwidth kernels."]
    with open(out, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print(out)


if __name__ == "__main__":
    main()
