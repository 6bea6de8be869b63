#!/bin/bash
# round 6: pinned-schedule register-blocked GEMM + fused run-routing slot maps, one GPU call
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py > gpurun_out/gemm_test.log 2>&1 || { echo "gemm tests failed"; tail -20 gpurun_out/gemm_test.log; exit 1; }
timeout -k 10 240 python -u tools/gemm_bench.py > gpurun_out/gemm_rb3.log 2>&1 || { echo "gemm bench failed"; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist1.py tests/test_gpu_shard.py tests/test_gpu_multiproc.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_rr.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_rr.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 --force_exchange > gpurun_out/proxy_$i.log 2>&1 || exit 1
  tail -1 gpurun_out/proxy_$i.log | cut -c1-200
done
bash scripts/prof_kernels.sh "r6px|--steps 20 --warmup 5 --force_exchange" > /dev/null || exit 1
