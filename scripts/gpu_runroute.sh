cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
true

for v in ; do
  t=${v%%|*}; envs=${v#*|}
  env $envs timeout -k 10 200 python bench.py --steps 100 --warmup 10 --force_exchange > gpurun_out/b_$t.log 2>&1 || exit $?
  echo "$t: $(tail -1 gpurun_out/b_$t.log | cut -c180-260)"
done
bash scripts/prof_kernels.sh "r3e_fx_run|--steps 100 --warmup 10 --force_exchange" > /dev/null
bash scripts/prof_kernels.sh "r3e_run|--steps 100 --warmup 10" > /dev/null
