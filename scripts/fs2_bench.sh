#!/bin/bash
# Standalone run-sort timing (tools/fsbench/fs2_bench.hip, built in-tree beforehand): full passes
# and pass-capped builds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for b in fs2b fs2b_p0 fs2b_p1 fs2b_p2; do
  echo "== $b"; timeout -k 5 60 tools/fsbench/$b || exit $?
done > gpurun_out/fs2_bench.log 2>&1
cat gpurun_out/fs2_bench.log
