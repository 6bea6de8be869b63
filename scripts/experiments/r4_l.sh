#!/bin/bash
# Replicated run-level routing (tests + Kaggle mode sweep) and the streamed path with two copy streams.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r4l}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_determinism.py > gpurun_out/${TAG}_pytest0.log 2>&1; rc=$?
fatal $rc pytest0
echo "pytest kernels/determinism rc=$rc: $(tail -1 gpurun_out/${TAG}_pytest0.log)"
[ $rc -ne 0 ] && { grep -E "Error|FAILED" gpurun_out/${TAG}_pytest0.log | head -10; exit $rc; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dist1.py tests/test_gpu_shard.py tests/test_gpu_e2e.py -k "replicated or streamed or run_routing or tf1_split" > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
fatal $rc pytest
echo "pytest rc=$rc: $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -ne 0 ] && { grep -E "Error|FAILED" gpurun_out/${TAG}_pytest.log | head -10; exit $rc; }
bash scripts/experiments/r4_modes.sh ${TAG}m; rc=$?; fatal $rc modes
for k in 1 2; do
  timeout -k 10 300 python bench.py --preset reference --embedding_size 32 --batch_size 1024 --steps 100 --warmup 5 > gpurun_out/${TAG}_ref.log 2>&1; rc=$?; fatal $rc ref
  echo "ref lazy: $(tail -1 gpurun_out/${TAG}_ref.log | grep -o '"ms_per_step": [0-9.]*')"
done
timeout -k 10 300 python bench.py --preset reference --embedding_size 32 --batch_size 1024 --steps 100 --warmup 5 --sparse_update tf1_dense > gpurun_out/${TAG}_ref_tf1.log 2>&1; rc=$?; fatal $rc ref_tf1
echo "ref tf1: $(tail -1 gpurun_out/${TAG}_ref_tf1.log | grep -o '"ms_per_step": [0-9.]*')"
L=$PWD/deepfm-tensorflow-distributed-training-on-sagemaker_amd/_lib
for k in 1 2; do
  for so in $L/libhipfm_kernels.so $L/libhipfm_kernels_wl.so; do
    [ -f $so ] || continue
    HIPFM_KERNELS_SO=$so timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_wl.log 2>&1; rc=$?; fatal $rc wl
    echo "$(basename $so) run $k: $(tail -1 gpurun_out/${TAG}_wl.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
bash scripts/stream_prof.sh ${TAG}s 4000000; rc=$?; fatal $rc stream
exit 0
