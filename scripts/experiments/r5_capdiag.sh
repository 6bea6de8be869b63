#!/bin/bash
# the streamed-ring capture failure after test_gpu_dx0_split.py: HIP's own log of the call that
# invalidated the capture (AMD_LOG_LEVEL=2: errors + warnings)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
E2E=tests/test_gpu_e2e.py::test_streamed_epochs_through_the_ring_train_like_the_cached_run
AMD_LOG_LEVEL=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_dx0_split.py $E2E -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/capd_full.log 2>&1
rc=$?; echo "rc=$rc $(tail -1 gpurun_out/capd_full.log)"
grep -n -i "captur\|invalid\|error" gpurun_out/capd_full.log | grep -v "^.*test_gpu" | head -30
