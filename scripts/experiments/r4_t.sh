#!/bin/bash
# dX0 launch with primed W_0 fragments: bitwise test, reference workload (lazy + tf1_dense) and
# headline benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r4t}
fatal() { case $1 in 0) ;; 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; *) echo "rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dx0_split.py > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_pytest.log; fatal $rc pytest
for k in 1 2; do
  timeout -k 10 300 python bench.py --preset reference --embedding_size 32 --batch_size 1024 --steps 100 --warmup 5 > gpurun_out/${TAG}_ref.log 2>&1; fatal $? ref
  echo "ref lazy run $k: $(tail -1 gpurun_out/${TAG}_ref.log | grep -o '"ms_per_step": [0-9.]*')"
  timeout -k 10 300 python bench.py --preset reference --embedding_size 32 --batch_size 1024 --steps 100 --warmup 5 --sparse_update tf1_dense > gpurun_out/${TAG}_ref_tf1.log 2>&1; fatal $? ref_tf1
  echo "ref tf1_dense run $k: $(tail -1 gpurun_out/${TAG}_ref_tf1.log | grep -o '"ms_per_step": [0-9.]*')"
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2>&1; fatal $? bench
  echo "bench run $k: $(tail -1 gpurun_out/${TAG}_bench.log | grep -o '"ms_per_step": [0-9.]*')"
done
timeout -k 10 400 bash scripts/prof_kernels.sh "${TAG}_ref|--preset reference --embedding_size 32 --batch_size 1024 --steps 64 --warmup 5"; fatal $? prof
sed -n '/One steady-state/,/step span/p' gpurun_out/${TAG}_ref_kernels.md
exit 0
