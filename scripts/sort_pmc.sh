#!/bin/bash
# Run-level sort microbenchmark + one PMC pass over it (gpurun_out/pmc_sort).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_sort
timeout -k 10 120 python3 tools/bench_sort.py --run > gpurun_out/sort_run.log 2>&1 || exit $?
timeout -k 10 120 python3 tools/bench_launch.py --xstream >> gpurun_out/sort_run.log 2>&1 || exit $?
cat gpurun_out/sort_run.log
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES --kernel-trace --stats --output-format csv \
  -d "$ROOT/gpurun_out/pmc_sort" -o run -- python3 "$ROOT/tools/bench_sort.py" --run > gpurun_out/pmc_sort/log.txt 2>&1
rc=$?; echo "pmc rc=$rc"
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pmc_sort/**/*counter_collection.csv", recursive=True)
if not f: raise SystemExit("no counter csv")
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f[0])):
    k = r["Kernel_Name"][:40]
    if "fs" not in k: continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
with open("gpurun_out/pmc_sort/summary.txt", "w") as o:
    for k, d in acc.items():
        line = k + ": " + ", ".join(f"{c}={v / max(1, n[(k, c)]):.3g}" for c, v in sorted(d.items()))
        print(line); o.write(line + "\n")
PY
