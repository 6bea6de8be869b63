#!/bin/bash
# 5 waves / SIMD merged launch (now the default) vs no attribute (w0): kernels + determinism
# tests, 3 headline benches each, Kaggle lazy + tf1 (K = 8), timeline of the default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r4zz}
fatal() { case $1 in 0) ;; 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; *) echo "rc=$1 at $2"; exit $1;; esac; }
L=$PWD/deepfm-tensorflow-distributed-training-on-sagemaker_amd/_lib
for t in test_gpu_determinism test_gpu_kernels test_gpu_tf1 test_gpu_run_sort; do
  timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/$t.py > gpurun_out/${TAG}_$t.log 2>&1; rc=$?
  echo "$t: $(tail -1 gpurun_out/${TAG}_$t.log)"; fatal $rc $t
done
for k in 1 2 3; do
  for v in base w0; do
    so=$L/libhipfm_kernels_$v.so; [ $v = base ] && so=$L/libhipfm_kernels.so
    HIPFM_KERNELS_SO=$so timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_$v.log 2>&1; fatal $? bench_$v
    echo "bench $v run $k: $(tail -1 gpurun_out/${TAG}_bench_$v.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
for v in base w0; do
  so=$L/libhipfm_kernels_$v.so; [ $v = base ] && so=$L/libhipfm_kernels.so
  HIPFM_KERNELS_SO=$so timeout -k 10 300 python bench.py --preset criteo_kaggle --steps 50 --warmup 5 > gpurun_out/${TAG}_kag_$v.log 2>&1; fatal $? kag_$v
  echo "kaggle lazy $v: $(tail -1 gpurun_out/${TAG}_kag_$v.log | grep -o '"ms_per_step": [0-9.]*')"
  HIPFM_KERNELS_SO=$so timeout -k 10 300 python bench.py --preset criteo_kaggle --steps 50 --warmup 5 --sparse_update tf1_dense > gpurun_out/${TAG}_kagt_$v.log 2>&1; fatal $? kagt_$v
  echo "kaggle tf1 $v: $(tail -1 gpurun_out/${TAG}_kagt_$v.log | grep -o '"ms_per_step": [0-9.]*')"
done
timeout -k 10 400 bash scripts/prof_kernels.sh "${TAG}_head|--steps 20 --warmup 5"; fatal $? prof
grep -A8 "One steady-state" gpurun_out/${TAG}_head_kernels.md
exit 0
