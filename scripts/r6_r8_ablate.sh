#!/bin/bash
# tile 13 ablations (timing only, wrong results): variant libraries built with HIPFM_BUILD_VARIANT
# (pure: no in-loop DMA, fragment reads or barriers; nodma: no in-loop DMA)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$(pwd)/deepfm-tensorflow-distributed-training-on-sagemaker_amd/_lib
for v in base ${VARIANTS:-pure nodma}; do
  if [ $v = base ]; then so=$L/libhipfm_kernels.so; else so=$L/libhipfm_kernels_$v.so; fi
  HIPFM_KERNELS_SO=$so timeout -k 10 200 python -u tools/gemm_bench.py --batch 4096 --width 4096 > gpurun_out/abl_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/abl_$v.log; exit 1; }
  echo "$v $(grep fwd_layer1 gpurun_out/abl_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["tile13_r8"]["tflops_median"], d["torch_matmul"]["tflops_median"])')"
done
