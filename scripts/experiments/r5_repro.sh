#!/bin/bash
# Round 5: the driver's one-process GPU suite without -x (every failure listed), then the n8
# test alone in a fresh process for comparison.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/r5a_pytest_all.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5a_pytest_all.log | tail -20
if [ $rc -ge 2 ]; then exit $rc; fi
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py -v -m gpu -k n8 --timeout 200 --timeout-method thread \
  > gpurun_out/r5a_pytest_n8.log 2>&1
echo "n8 alone rc=$?"; tail -3 gpurun_out/r5a_pytest_n8.log
