#!/bin/bash
# One GPU call: all GPU tests (one process), smoke, then the benches given as arguments
# ("ENV=.. ENV2=.. -- bench args" strings).  Every GPU step has its own time limit and the script
# stops at the first failure (no retries).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ]; then exit $rc; fi
  timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
i=0
for spec in "$@"; do
  i=$((i + 1))
  # "ENV=a ENV2=b -- bench args" or just "bench args"
  case "$spec" in
    *" -- "*) envs="${spec%% -- *}"; args="${spec#* -- }" ;;
    *) envs=""; args="$spec" ;;
  esac
  echo "bench[$i] env=[$envs] args=[$args]"
  env $envs timeout -k 10 300 python bench.py $args > gpurun_out/bench_$i.log 2>&1
  rc=$?; tail -1 gpurun_out/bench_$i.log
  if [ $rc -ne 0 ]; then echo "bench[$i] rc=$rc"; exit $rc; fi
done
