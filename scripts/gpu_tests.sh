#!/bin/bash
# All GPU-marked tests in ONE process (the box allows few GPU processes), then smoke.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ge 2 ]; then exit $rc; fi
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc2=$?; echo "smoke rc=$rc2"; tail -2 gpurun_out/smoke.log
if [ $rc2 -ne 0 ]; then exit $rc2; fi
exit $rc
