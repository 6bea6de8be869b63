#!/bin/bash
# K <= 16 sparse tile size A/B on the headline (512 vs 256 slots; variant library HFM_SF_TP8=256)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$(pwd)/deepfm-tensorflow-distributed-training-on-sagemaker_amd/_lib
for rep in 1 2 3; do
  for v in base tp256; do
    if [ $v = base ]; then so=$L/libhipfm_kernels.so; else so=$L/libhipfm_kernels_$v.so; fi
    HIPFM_KERNELS_SO=$so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/tp8_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/tp8_$v.log; exit 1; }
    echo "$v $(tail -1 gpurun_out/tp8_$v.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
