#!/bin/bash
# Round 5: the rank-stream wait fix -- its regression test alone, then the driver-shaped suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_shard.py -q -m gpu -k "rank_streams_wait" --timeout 150 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r5i_regress.log 2>&1
echo "regress rc=$? $(tail -1 gpurun_out/r5i_regress.log)"
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r5i_pytest_gpu.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r5i_pytest_gpu.log
exit $rc
