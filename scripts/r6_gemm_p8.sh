#!/bin/bash
# round 6: K-half ring GEMM (tile 12) correctness + throughput, fused run-routing scatter proxy
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py > gpurun_out/gemm_test.log 2>&1 || { echo "gemm tests failed"; tail -30 gpurun_out/gemm_test.log; exit 1; }
timeout -k 10 300 python -u tools/gemm_bench.py > gpurun_out/gemm_p8.log 2>&1 || { echo "gemm bench failed"; tail gpurun_out/gemm_p8.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist1.py tests/test_gpu_shard.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_rr.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_rr.log; [ $rc -ne 0 ] && exit $rc
bash scripts/prof_kernels.sh "r6px2|--steps 20 --warmup 5 --force_exchange" > /dev/null || exit 1
