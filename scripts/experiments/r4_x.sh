#!/bin/bash
# dX0 launch with the block's sorted positions staged in LDS: its test, the reference workload,
# and the timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r4x}
fatal() { case $1 in 0) ;; 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; *) echo "rc=$1 at $2"; exit $1;; esac; }
for t in test_gpu_dx0_split test_gpu_run_sort; do
  timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/$t.py > gpurun_out/${TAG}_$t.log 2>&1; rc=$?
  echo "$t: $(tail -1 gpurun_out/${TAG}_$t.log)"; fatal $rc $t
done
R="--preset reference --embedding_size 32 --batch_size 1024 --steps 100 --warmup 5"
for k in 1 2; do
  timeout -k 10 300 python bench.py $R > gpurun_out/${TAG}_ref.log 2>&1; fatal $? ref
  echo "ref lazy run $k: $(tail -1 gpurun_out/${TAG}_ref.log | grep -o '"ms_per_step": [0-9.]*')"
  timeout -k 10 300 python bench.py $R --sparse_update tf1_dense > gpurun_out/${TAG}_ref_tf1.log 2>&1; fatal $? ref_tf1
  echo "ref tf1 run $k: $(tail -1 gpurun_out/${TAG}_ref_tf1.log | grep -o '"ms_per_step": [0-9.]*')"
done
timeout -k 10 400 bash scripts/prof_kernels.sh "${TAG}_ref|--preset reference --embedding_size 32 --batch_size 1024 --steps 64 --warmup 5"; fatal $? prof
grep -A9 "One steady-state" gpurun_out/${TAG}_ref_kernels.md
exit 0
