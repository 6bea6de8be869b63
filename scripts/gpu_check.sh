#!/bin/bash
# GPU-box validation: kernel numerics tests, smoke, short benches.  Each GPU step has its own
# time limit; a crash / abort / timeout (rc >= 2 for pytest, != 0 otherwise) stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HIP_LAUNCH_BLOCKING=${HIP_LAUNCH_BLOCKING:-0}
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ge 2 ]; then exit $rc; fi
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
for args in "$@"; do
  echo "bench $args"
  timeout -k 10 600 python bench.py $args > gpurun_out/bench_$(echo $args | tr ' -' '_').log 2>&1
  rc=$?; tail -2 gpurun_out/bench_$(echo $args | tr ' -' '_').log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
