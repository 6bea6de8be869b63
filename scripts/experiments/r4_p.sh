#!/bin/bash
# Reference workload A/B: the sparse tile's early record load at K = 32 on (pa) or off (base);
# headline driver-window benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r4p}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
L=$PWD/deepfm-tensorflow-distributed-training-on-sagemaker_amd/_lib
for k in 1 2 3; do
  for v in base pa; do
    so=$L/libhipfm_kernels_$v.so; [ $v = base ] && so=$L/libhipfm_kernels.so
    [ -f $so ] || continue
    HIPFM_KERNELS_SO=$so timeout -k 10 300 python bench.py --preset reference --embedding_size 32 --batch_size 1024 --steps 100 --warmup 5 > gpurun_out/${TAG}_ref.log 2>&1; rc=$?; fatal $rc ref_$v
    echo "ref $v run $k: $(tail -1 gpurun_out/${TAG}_ref.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
for k in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench$k.log 2>&1; rc=$?; fatal $rc bench
  echo "bench $k: $(tail -1 gpurun_out/${TAG}_bench$k.log | grep -o '"ms_per_step": [0-9.]*')"
done
exit 0
