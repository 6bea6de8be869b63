#!/bin/bash
# dX0 launch: dZ_0 transposed into LDS two rows per item (4-B writes, base) vs one (d1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r4d1}
fatal() { case $1 in 0) ;; 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; *) echo "rc=$1 at $2"; exit $1;; esac; }
L=$PWD/deepfm-tensorflow-distributed-training-on-sagemaker_amd/_lib
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dx0_split.py > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "dx0 tests: $(tail -1 gpurun_out/${TAG}_pytest.log)"; fatal $rc pytest
R="--preset reference --embedding_size 32 --batch_size 1024 --steps 100 --warmup 5"
for k in 1 2 3; do
  for v in base d1; do
    so=$L/libhipfm_kernels_$v.so; [ $v = base ] && so=$L/libhipfm_kernels.so
    HIPFM_KERNELS_SO=$so timeout -k 10 300 python bench.py $R > gpurun_out/${TAG}_ref_$v.log 2>&1; fatal $? ref_$v
    echo "ref $v run $k: $(tail -1 gpurun_out/${TAG}_ref_$v.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
exit 0
