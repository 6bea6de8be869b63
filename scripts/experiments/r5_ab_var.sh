#!/bin/bash
# timing-only kernel variants (numerically wrong): usage r5_ab_var.sh TAG1 TAG2 ... (base first)
cd $GRAFT_REPO_ROOT
L=$GRAFT_REPO_ROOT/deepfm-tensorflow-distributed-training-on-sagemaker_amd/_lib
for i in 1 2 3 4 5; do
  for t in base "$@"; do
    if [ $t = base ]; then so=$L/libhipfm_kernels.so; else so=$L/libhipfm_kernels_$t.so; fi
    HIPFM_KERNELS_SO=$so timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/var_${t}_$i.log 2>&1
    echo "$t $(tail -1 gpurun_out/var_${t}_$i.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])' 2>&1 | tail -1)"
  done
done
