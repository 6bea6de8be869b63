#!/bin/bash
# Kaggle-shape step times across the execution modes (1 GPU; the exchange modes as 1-rank
# proxies): local / replicated / row-sharded x lazy / tf1_dense.  usage: scripts/experiments/r4_modes.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-modes}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --preset criteo_kaggle --steps 50 --warmup 5 "$@" > gpurun_out/${TAG}_$name.log 2>&1; local rc=$?
  fatal $rc $name
  echo "$name rc=$rc: $(tail -1 gpurun_out/${TAG}_$name.log | python -c 'import json,sys
try:
  d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["parallelism"], d["eval_auc"])
except Exception as e: print("?", e)')"
}
run local_lazy --sparse_update lazy
run repl_lazy --sparse_update lazy --force_exchange --embedding_mode replicated
run shard_lazy --sparse_update lazy --force_exchange --embedding_mode sharded
run local_tf1 --sparse_update tf1_dense
run repl_tf1 --sparse_update tf1_dense --force_exchange --embedding_mode replicated
run shard_tf1 --sparse_update tf1_dense --force_exchange --embedding_mode sharded
exit 0
