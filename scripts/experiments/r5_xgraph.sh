#!/bin/bash
# 1-rank proxy: steps per captured multi-rank graph (the driver's 20-step window)
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for g in 16 20 32; do
    HIPFM_BENCH_XGRAPH=$g timeout -k 10 300 python bench.py --steps 20 --warmup 5 --force_exchange > gpurun_out/r5y_g${g}_$i.log 2>&1
    echo "xgraph=$g rc=$? $(tail -1 gpurun_out/r5y_g${g}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["graph_steps"], d["config"]["exec"])' 2>&1 | tail -1)"
  done
done
