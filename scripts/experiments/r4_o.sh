#!/bin/bash
# Resume (skip) through the streamed ring: the fault test and the e2e tests, then the reference
# workload A/B over the K = 32 tower variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r4o}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_gpu_fault.py tests/test_gpu_e2e.py > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
fatal $rc pytest
echo "pytest rc=$rc: $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -ne 0 ] && { grep -E "^FAILED|Timeout" gpurun_out/${TAG}_pytest.log | head -10; exit $rc; }
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
