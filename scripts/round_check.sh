#!/bin/bash
# Round-end check in the DRIVER's shape: ONE `pytest -m gpu -x` process over the whole suite (a
# per-file runner hides state that survives between tests -- the round-4 n8 failure), then the
# smoke, then the 1-GPU bench line exactly as the driver invokes it.  Every GPU step has its own
# time limit and the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-rc}
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; echo "pytest -m gpu rc=$rc: $(tail -1 gpurun_out/${TAG}_pytest_gpu.log)"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc: $(tail -1 gpurun_out/${TAG}_smoke.log)"
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_$i.log 2>&1
  rc=$?; echo "bench[$i] rc=$rc: $(tail -1 gpurun_out/${TAG}_bench_$i.log)"
  [ $rc -eq 0 ] || exit $rc
done
