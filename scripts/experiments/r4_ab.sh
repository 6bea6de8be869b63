#!/bin/bash
# A/B of bench configurations (env prefixes) in one GPU call: kernel trace summary per arm
# (gpurun_out/<tag>_<i>_kernels.md) + the bench line, then the stamp profile of the first arm.
# usage: scripts/r4_ab.sh <tag> "<env for arm 1>" "<env for arm 2>" ... (bench args in $BARGS)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=$1; shift
A="${BARGS:---steps 20 --warmup 5}"
i=0
for envs in "$@"; do
  i=$((i + 1))
  env $envs bash scripts/profile.sh "${TAG}_$i" $A || exit $?
  python tools/prof_summary.py "gpurun_out/prof_${TAG}_$i" "gpurun_out/${TAG}_${i}_kernels.md" "$TAG arm $i ($envs): bench $A" > /dev/null || exit $?
  rm -rf "gpurun_out/prof_${TAG}_$i"
  env $envs timeout -k 10 300 python bench.py $A > gpurun_out/${TAG}_${i}_bench.log 2>&1 || exit $?
  echo "arm $i ($envs): $(tail -1 gpurun_out/${TAG}_${i}_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("eval_auc"))')"
done
