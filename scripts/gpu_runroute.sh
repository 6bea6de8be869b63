cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist1.py tests/test_gpu_shard.py -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_rr.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_rr.log; [ $rc -ne 0 ] && exit $rc
bash scripts/prof_kernels.sh "r3e_fx_run|--steps 100 --warmup 10 --force_exchange" > /dev/null
echo "$(sed -n 6p gpurun_out/r3e_fx_run_kernels.md | cut -c180-260)"
