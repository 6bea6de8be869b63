#!/bin/bash
# counter-rank vs ballot run-sort body (tools/fsbench/fs2_bench.hip)
set -o pipefail
mkdir -p gpurun_out
cd tools/fsbench && hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../csrc/kernels fs2_bench.hip -o fs2b 2>/dev/null && cd ../.. \
  && FS2_QUICK=1 timeout -k 10 120 tools/fsbench/fs2b > gpurun_out/r4q_fs2.log 2>&1
rc=$?; cat gpurun_out/r4q_fs2.log | tail -80; exit $rc
