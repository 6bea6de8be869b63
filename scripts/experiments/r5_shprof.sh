#!/bin/bash
# row-sharded proxies: Criteo-1TB headline shape (lazy) and Kaggle tf1_dense, kernel traces
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r5s_1tb -o run -- \
  python3 bench.py --steps 20 --warmup 5 --force_exchange > gpurun_out/prof_r5s_1tb.log 2>&1 || { echo "prof 1tb failed"; exit 1; }
tail -1 gpurun_out/prof_r5s_1tb.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r5s_tf1 -o run -- \
  python3 bench.py --preset criteo_kaggle --steps 50 --warmup 5 --sparse_update tf1_dense --force_exchange \
  --embedding_mode sharded > gpurun_out/prof_r5s_tf1.log 2>&1 || { echo "prof tf1 failed"; exit 1; }
tail -1 gpurun_out/prof_r5s_tf1.log | cut -c1-200
