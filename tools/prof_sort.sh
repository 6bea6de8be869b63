#!/bin/bash
# Kernel-level profile of the id sorts (graph replays) -> gpurun_out/prof_sort/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_sort
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sort -o run -- python3 tools/bench_sort.py --only 638976 > gpurun_out/prof_sort/bench.log 2>&1
echo "rocprof rc=$?"
