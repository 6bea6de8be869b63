#!/bin/bash
# Standalone run-sort timing and correctness (tools/fsbench/fs2_bench.hip): the counter-rank form
# against the ballot form over field widths, batch sizes and id layouts, each checked against
# std::stable_sort.  Build it on the CPU first:
#   (cd tools/fsbench && hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../csrc/kernels fs2_bench.hip -o fs2b)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
FS2_QUICK=1 timeout -k 5 120 tools/fsbench/fs2b > gpurun_out/fs2_bench.log 2>&1; rc=$?
tail -5 gpurun_out/fs2_bench.log
exit $rc
