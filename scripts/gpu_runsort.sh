cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_run_sort.py -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_runsort.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_runsort.log; [ $rc -ne 0 ] && exit $rc
for v in "run|HIPFM_RUN_SORT=1" "side|HIPFM_RUN_SORT=0" "runfm|HIPFM_RUN_SORT=1 --field_major_ids"; do
  t=${v%%|*}; rest=${v#*|}; envs=${rest%% --*}; args=""; case "$rest" in *" --"*) args="--${rest#* --}";; esac
  env $envs timeout -k 10 200 python bench.py --steps 100 --warmup 10 $args > gpurun_out/b_$t.log 2>&1 || exit $?
  echo "$t: $(tail -1 gpurun_out/b_$t.log | cut -c180-260)"
done
timeout -k 10 200 python bench.py --steps 20 --warmup 10 > gpurun_out/b_run20.log 2>&1 || exit $?
echo "run20: $(tail -1 gpurun_out/b_run20.log | cut -c180-260)"
bash scripts/prof_kernels.sh "r3d_run|--steps 100 --warmup 10" > /dev/null
