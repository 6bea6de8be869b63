#!/bin/bash
# Round 5: is the n8 pass due to the rank-stream wait, or to the test order the new test changed?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local lab=$1; shift
  timeout -k 10 400 python -u -m pytest tests -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider "$@" \
    > gpurun_out/r5k_$lab.log 2>&1
  local rc=$?
  echo "$lab rc=$rc $(tail -1 gpurun_out/r5k_$lab.log)"; grep FAILED gpurun_out/r5k_$lab.log | head -3
  [ $rc -le 1 ]
}
R5_NOWAIT=1 run nowait_with_regress || exit 1
run wait_without_regress -k "not rank_streams_wait" || exit 1
R5_NOWAIT=1 run nowait_without_regress -k "not rank_streams_wait" || exit 1
