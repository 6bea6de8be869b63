#!/bin/bash
# Full GPU test suite, then the reference workload (B = 1024, K = 32) A/B over the K = 32 tower
# variants and its stamps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r4m}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
fatal $rc pytest
echo "pytest rc=$rc: $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -ne 0 ] && grep -E "^FAILED|^ERROR" gpurun_out/${TAG}_pytest.log | head -10
L=$PWD/deepfm-tensorflow-distributed-training-on-sagemaker_amd/_lib
for k in 1 2; do
  for v in base f2 dd old; do
    so=$L/libhipfm_kernels_$v.so; [ $v = base ] && so=$L/libhipfm_kernels.so
    [ -f $so ] || continue
    HIPFM_KERNELS_SO=$so timeout -k 10 300 python bench.py --preset reference --embedding_size 32 --batch_size 1024 --steps 100 --warmup 5 > gpurun_out/${TAG}_ref.log 2>&1; rc=$?; fatal $rc ref_$v
    echo "ref $v run $k: $(tail -1 gpurun_out/${TAG}_ref.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
exit 0
