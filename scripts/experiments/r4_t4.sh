#!/bin/bash
# Transposed tile stores of 4 columns per thread (base) vs 1 (t1): affected tests, headline and
# reference-workload benches, timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r4t4}
fatal() { case $1 in 0) ;; 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; *) echo "rc=$1 at $2"; exit $1;; esac; }
L=$PWD/deepfm-tensorflow-distributed-training-on-sagemaker_amd/_lib
for t in test_gpu_kernels test_gpu_determinism test_gpu_dx0_split test_gpu_fp8 test_gpu_shard; do
  timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/$t.py > gpurun_out/${TAG}_$t.log 2>&1; rc=$?
  echo "$t: $(tail -1 gpurun_out/${TAG}_$t.log)"; fatal $rc $t
done
R="--preset reference --embedding_size 32 --batch_size 1024 --steps 100 --warmup 5"
for k in 1 2 3; do
  for v in base t1; do
    so=$L/libhipfm_kernels_$v.so; [ $v = base ] && so=$L/libhipfm_kernels.so
    HIPFM_KERNELS_SO=$so timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_$v.log 2>&1; fatal $? bench_$v
    echo "bench $v run $k: $(tail -1 gpurun_out/${TAG}_bench_$v.log | grep -o '"ms_per_step": [0-9.]*')"
    HIPFM_KERNELS_SO=$so timeout -k 10 300 python bench.py $R > gpurun_out/${TAG}_ref_$v.log 2>&1; fatal $? ref_$v
    echo "ref $v run $k: $(tail -1 gpurun_out/${TAG}_ref_$v.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
timeout -k 10 400 bash scripts/prof_kernels.sh "${TAG}_head|--steps 20 --warmup 5" "${TAG}_ref|--preset reference --embedding_size 32 --batch_size 1024 --steps 64 --warmup 5"; fatal $? prof
grep -A9 "One steady-state" gpurun_out/${TAG}_head_kernels.md gpurun_out/${TAG}_ref_kernels.md
exit 0
