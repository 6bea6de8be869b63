#!/bin/bash
# Round 5: cumulative prefixes of the one-process GPU suite, each followed by the n8 test.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N8=tests/test_gpu_shard.py::test_sharded_exchange_n8_criteo_1tb_shape
run() {
  local lab=$1; shift
  timeout -k 10 400 python -u -m pytest "$@" -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r5f_$lab.log 2>&1
  local rc=$?
  echo "$lab rc=$rc $(tail -1 gpurun_out/r5f_$lab.log)"
  [ $rc -le 1 ]
}
T=tests/test_gpu_
ALL="${T}bn.py ${T}determinism.py ${T}dist1.py ${T}dx0_split.py ${T}e2e.py ${T}fault.py ${T}fp8.py ${T}kernels.py ${T}mixed.py ${T}plan_state.py ${T}run_sort.py ${T}safety.py"

run D $ALL ${T}shard.py || exit 1
