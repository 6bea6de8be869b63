#!/bin/bash
# Counter-rank run sort: sort tests, then A/B against the ballot-rank build (bl) on the headline
# and reference-workload benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r4r}
fatal() { case $1 in 0) ;; 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; *) echo "rc=$1 at $2";; esac; }
L=$PWD/deepfm-tensorflow-distributed-training-on-sagemaker_amd/_lib
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_run_sort.py tests/test_gpu_dx0_split.py > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_pytest.log; [ $rc = 0 ] || { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "sort" > gpurun_out/${TAG}_pytest2.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_pytest2.log; [ $rc = 0 ] || { echo "pytest2 rc=$rc"; exit $rc; }
for k in 1 2; do
  for v in base bl; do
    so=$L/libhipfm_kernels_$v.so; [ $v = base ] && so=$L/libhipfm_kernels.so
    HIPFM_KERNELS_SO=$so timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_$v.log 2>&1; rc=$?; fatal $rc bench_$v
    echo "bench $v run $k: $(tail -1 gpurun_out/${TAG}_bench_$v.log | grep -o '"ms_per_step": [0-9.]*')"
    HIPFM_KERNELS_SO=$so timeout -k 10 300 python bench.py --preset reference --embedding_size 32 --batch_size 1024 --steps 100 --warmup 5 > gpurun_out/${TAG}_ref_$v.log 2>&1; rc=$?; fatal $rc ref_$v
    echo "ref $v run $k: $(tail -1 gpurun_out/${TAG}_ref_$v.log | grep -o '"ms_per_step": [0-9.]*')"
  done
  HIPFM_DX0_SPLIT=0 timeout -k 10 300 python bench.py --preset reference --embedding_size 32 --batch_size 1024 --steps 100 --warmup 5 > gpurun_out/${TAG}_ref_nosplit.log 2>&1; rc=$?; fatal $rc ref_nosplit
  echo "ref nosplit run $k: $(tail -1 gpurun_out/${TAG}_ref_nosplit.log | grep -o '"ms_per_step": [0-9.]*')"
done
exit 0
