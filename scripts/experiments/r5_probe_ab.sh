#!/bin/bash
# owner update probing this step's and the next step's request tables together: sharded tests,
# then the 1-rank proxy alternating the previous library (abso/old_kernels.so) and this one
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shard.py tests/test_gpu_dist1.py \
  > gpurun_out/r5pb_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r5pb_tests.log; exit 1; }
tail -1 gpurun_out/r5pb_tests.log
for i in 1 2 3; do
  for v in old new; do
    so=""; [ $v = old ] && so=$GRAFT_REPO_ROOT/abso/old_kernels.so
    HIPFM_KERNELS_SO=$so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --force_exchange > gpurun_out/r5pb_${v}_$i.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/r5pb_${v}_$i.log; exit 1; }
    echo "$v run=$i $(tail -1 gpurun_out/r5pb_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["eval_auc"])')"
  done
done
