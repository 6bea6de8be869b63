#!/bin/bash
# One GPU call: driver-shaped bench (x2), the 1-rank sharded proxy with its kernel trace, a set of
# GPU test files, and (optionally) the file-fed data bench.  Stops at the first step that times
# out, aborts or faults (exit 124 / 134 / 137 / 139); a plain test failure does not stop the
# benches that follow.   usage: TESTS="tests/a.py ..." DATA=1 scripts/r4_round.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r4}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
for k in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench$k.log 2>&1; rc=$?
  fatal $rc bench$k
  echo "bench$k rc=$rc: $(tail -1 gpurun_out/${TAG}_bench$k.log | cut -c1-400)"
done
bash scripts/profile.sh "${TAG}_px" --steps 20 --warmup 5 --force_exchange > /dev/null 2>&1; rc=$?; fatal $rc proxy
python tools/prof_summary.py "gpurun_out/prof_${TAG}_px" "gpurun_out/${TAG}_px_kernels.md" "$TAG: bench --force_exchange" > /dev/null
rm -rf "gpurun_out/prof_${TAG}_px"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --force_exchange > gpurun_out/${TAG}_px.log 2>&1; rc=$?
fatal $rc proxy_bench
echo "proxy rc=$rc: $(tail -1 gpurun_out/${TAG}_px.log | cut -c1-300)"
if [ -n "$TESTS" ]; then
  timeout -k 10 1200 python -u -m pytest -v --timeout 300 --timeout-method thread $TESTS > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
  fatal $rc pytest
  echo "pytest rc=$rc: $(tail -1 gpurun_out/${TAG}_pytest.log)"
  grep -E "FAILED|ERROR" gpurun_out/${TAG}_pytest.log | head -20
fi
if [ -n "$DATA" ]; then
  bash scripts/data_bench.sh 2000000 --epochs 3; rc=$?; fatal $rc data
fi
exit 0
