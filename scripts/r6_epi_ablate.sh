#!/bin/bash
# tile 10 with / without its epilogue (timing only): how much of a wide-layer GEMM is the epilogue
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$(pwd)/deepfm-tensorflow-distributed-training-on-sagemaker_amd/_lib
for v in base noepi; do
  if [ $v = base ]; then so=$L/libhipfm_kernels.so; else so=$L/libhipfm_kernels_$v.so; fi
  for shp in "--batch 16384 --width 4096" "--batch 4096 --width 4096"; do
    HIPFM_KERNELS_SO=$so timeout -k 10 200 python -u tools/gemm_bench.py $shp > gpurun_out/epi_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/epi_$v.log; exit 1; }
    echo "$v $shp $(python -c 'import json,sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d=json.loads(l); print(d["shape"], d["tile10_pp3"]["tflops_median"], d["torch_matmul"]["tflops_median"], end=" | ")' gpurun_out/epi_$v.log)"
  done
done
