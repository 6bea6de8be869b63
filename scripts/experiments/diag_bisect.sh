cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for mods in "tests/test_gpu_safety.py" "tests/test_gpu_kernels.py" "tests/test_gpu_e2e.py tests/test_gpu_fp8.py" "tests/test_gpu_bn.py tests/test_gpu_determinism.py tests/test_gpu_dist1.py"; do
  timeout -k 10 400 python -u -m pytest $mods tests/test_gpu_shard.py -q -k "not replicated and not collective and not two_launch" --timeout 200 --timeout-method thread > gpurun_out/bis.log 2>&1
  rc=$?
  echo "[$mods] rc=$rc $(tail -1 gpurun_out/bis.log)"; grep "max|dv|" gpurun_out/bis.log | grep "^E" | head -1
  if [ $rc -ge 2 ]; then exit $rc; fi
done
