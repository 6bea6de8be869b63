#!/bin/bash
# Round 5: which earlier GPU test file leaves process state that breaks the n8 sharded test?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N8=tests/test_gpu_shard.py::test_sharded_exchange_n8_criteo_1tb_shape
run() {  # $1 = label, rest = pytest args
  local lab=$1; shift
  timeout -k 10 300 python -u -m pytest "$@" -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r5b_$lab.log 2>&1
  local rc=$?
  echo "$lab rc=$rc $(tail -1 gpurun_out/r5b_$lab.log)"
  [ $rc -le 1 ]
}
run shard_file tests/test_gpu_shard.py || exit 1
for f in bn determinism dist1 dx0_split e2e fault fp8 kernels mixed plan_state run_sort safety; do
  run $f tests/test_gpu_$f.py $N8 || exit 1
done
