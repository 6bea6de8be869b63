#!/bin/bash
# 1-GPU bench over warm-up / step counts (the driver runs --steps 20 --warmup 5)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for v in "5 20" "10 20" "6 20" "5 21" "4 20" "5 20" "6 20" "4 20" "5 20"; do
  set -- $v
  timeout -k 10 200 python bench.py --steps $2 --warmup $1 > gpurun_out/w_$1_$2.log 2>&1 || exit $?
  echo "W=$1 K=$2: $(tail -1 gpurun_out/w_$1_$2.log | grep -o '"ms_per_step": [0-9.]*\|warmup_graph_captures": [0-9]*' | tr '\n' ' ')"
done
