#!/bin/bash
# the reference's own workload (B = 1024, K = 32): lazy and tf1_dense step times + tf1 kernel trace
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for u in lazy tf1_dense lazy tf1_dense; do
  timeout -k 10 300 python bench.py --preset reference --embedding_size 32 --batch_size 1024 --steps 64 --warmup 5 \
    --sparse_update $u > gpurun_out/r5r_$u.log 2>&1 || { echo "$u failed"; tail -5 gpurun_out/r5r_$u.log; exit 1; }
  echo "$u $(tail -1 gpurun_out/r5r_$u.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["eval_auc"])')"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r5r_tf1 -o run -- \
  python3 bench.py --preset reference --embedding_size 32 --batch_size 1024 --steps 64 --warmup 5 --sparse_update tf1_dense \
  > gpurun_out/prof_r5r_tf1.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
