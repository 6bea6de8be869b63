#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py > gpurun_out/gemm_test.log 2>&1 || { echo "gemm tests failed"; tail -30 gpurun_out/gemm_test.log; exit 1; }
timeout -k 10 300 python -u tools/gemm_bench.py > gpurun_out/gemm_p8b.log 2>&1 || { echo "gemm bench failed"; tail gpurun_out/gemm_p8b.log; exit 1; }
