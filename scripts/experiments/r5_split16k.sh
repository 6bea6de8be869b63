#!/bin/bash
# headline with the dX0 launch (and the layer-0 split it enables) forced on at B = 16384, A/B x3
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in default split; do
    env=""; [ $v = split ] && env="HIPFM_DX0_SPLIT=1"
    env $env timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r5sp_${v}_$i.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/r5sp_${v}_$i.log; exit 1; }
    echo "$v run=$i $(tail -1 gpurun_out/r5sp_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["eval_auc"])')"
  done
done
