#!/bin/bash
# Bench A/B over env arms, each arm run twice alternating (A B A B) to expose box noise, plus the
# kernel trace of the sharded proxy and an emb_dtype=bf16 bench.  Stops on a fatal exit code.
# usage: scripts/r4_ab2.sh <tag> "<env arm 1>" "<env arm 2>"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=$1; shift
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
for rep in 1 2; do
  i=0
  for envs in "$@"; do
    i=$((i + 1))
    env $envs timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_${i}_${rep}.log 2>&1; rc=$?
    fatal $rc "arm $i"
    echo "arm $i rep $rep ($envs): $(tail -1 gpurun_out/${TAG}_${i}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
bash scripts/profile.sh "${TAG}_px" --steps 20 --warmup 5 --force_exchange > /dev/null 2>&1; rc=$?; fatal $rc proxy
python tools/prof_summary.py "gpurun_out/prof_${TAG}_px" "gpurun_out/${TAG}_px_kernels.md" "$TAG: bench --force_exchange" > /dev/null
rm -rf "gpurun_out/prof_${TAG}_px"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --force_exchange > gpurun_out/${TAG}_px.log 2>&1; rc=$?; fatal $rc proxy_bench
echo "proxy: $(tail -1 gpurun_out/${TAG}_px.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["parallelism"], d.get("comm_bytes_per_step"), d.get("comm_bytes_moved_per_step"))')"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --emb_dtype bf16 > gpurun_out/${TAG}_bf16.log 2>&1; rc=$?; fatal $rc bf16
echo "emb bf16: $(tail -1 gpurun_out/${TAG}_bf16.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["eval_auc"])')"
