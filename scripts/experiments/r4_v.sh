#!/bin/bash
# Tower gather: next pass's ids prefetched (base) vs loaded at the pass start (np), reference
# workload lazy + tf1_dense and the headline; the dX0 split test and the tower numerics tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r4v}
fatal() { case $1 in 0) ;; 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; *) echo "rc=$1 at $2"; exit $1;; esac; }
L=$PWD/deepfm-tensorflow-distributed-training-on-sagemaker_amd/_lib
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dx0_split.py tests/test_gpu_determinism.py > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_pytest.log; fatal $rc pytest
R="--preset reference --embedding_size 32 --batch_size 1024 --steps 100 --warmup 5"
for k in 1 2; do
  for v in base np; do
    so=$L/libhipfm_kernels_$v.so; [ $v = base ] && so=$L/libhipfm_kernels.so
    HIPFM_KERNELS_SO=$so timeout -k 10 300 python bench.py $R > gpurun_out/${TAG}_ref_$v.log 2>&1; fatal $? ref_$v
    echo "ref lazy $v run $k: $(tail -1 gpurun_out/${TAG}_ref_$v.log | grep -o '"ms_per_step": [0-9.]*')"
    HIPFM_KERNELS_SO=$so timeout -k 10 300 python bench.py $R --sparse_update tf1_dense > gpurun_out/${TAG}_ref_tf1_$v.log 2>&1; fatal $? ref_tf1_$v
    echo "ref tf1 $v run $k: $(tail -1 gpurun_out/${TAG}_ref_tf1_$v.log | grep -o '"ms_per_step": [0-9.]*')"
  done
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2>&1; fatal $? bench
  echo "bench run $k: $(tail -1 gpurun_out/${TAG}_bench.log | grep -o '"ms_per_step": [0-9.]*')"
done
exit 0
