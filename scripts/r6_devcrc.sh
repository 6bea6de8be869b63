#!/bin/bash
# round 6: data CRCs on the GPU -- decode tests, streamed e2e bitwise test, streamed A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode.py "tests/test_gpu_e2e.py::test_streamed_epochs_through_the_ring_train_like_the_cached_run" > gpurun_out/devcrc_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/devcrc_tests.log; exit 1; }
tail -1 gpurun_out/devcrc_tests.log
ARMS="1 2 0" bash scripts/stream_decode_ab.sh 16000000 64 2 --epochs 3
