#!/bin/bash
# Merged sparse + wgfin launch at 5 waves / SIMD (w5: 8 spilled VGPRs) vs 4 (base): headline,
# reference workload; timeline of w5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r4y}
fatal() { case $1 in 0) ;; 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; *) echo "rc=$1 at $2"; exit $1;; esac; }
L=$PWD/deepfm-tensorflow-distributed-training-on-sagemaker_amd/_lib
R="--preset reference --embedding_size 32 --batch_size 1024 --steps 100 --warmup 5"
for k in 1 2; do
  for v in base w5 w5p1; do
    so=$L/libhipfm_kernels_$v.so; [ $v = base ] && so=$L/libhipfm_kernels.so
    HIPFM_KERNELS_SO=$so timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_$v.log 2>&1; fatal $? bench_$v
    echo "bench $v run $k: $(tail -1 gpurun_out/${TAG}_bench_$v.log | grep -o '"ms_per_step": [0-9.]*')"
    HIPFM_KERNELS_SO=$so timeout -k 10 300 python bench.py $R > gpurun_out/${TAG}_ref_$v.log 2>&1; fatal $? ref_$v
    echo "ref $v run $k: $(tail -1 gpurun_out/${TAG}_ref_$v.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
HIPFM_KERNELS_SO=$L/libhipfm_kernels_w5p1.so timeout -k 10 400 bash scripts/prof_kernels.sh "${TAG}_w5p1|--steps 20 --warmup 5"; fatal $? prof
grep -A8 "One steady-state" gpurun_out/${TAG}_w5p1_kernels.md
exit 0
