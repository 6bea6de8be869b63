#!/bin/bash
# tf1_dense split-sweep checks: the bitwise GPU tests, then the Kaggle-shape bench per sweep mode.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tf1.py -v -m gpu -x --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_tf1.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_tf1.log
[ $rc -ne 0 ] && exit $rc
for spec in "HIPFM_SWEEP_MODE=auto" "HIPFM_SWEEP_MODE=merged" "HIPFM_SWEEP_MODE=branch" "HIPFM_TF1_SPLIT=0"; do
  env $spec timeout -k 10 200 python bench.py --preset criteo_kaggle --sparse_update tf1_dense --steps 300 \
    --warmup 30 > gpurun_out/tf1_b.log 2>&1 || exit $?
  echo "$spec"; tail -1 gpurun_out/tf1_b.log | cut -c150-200
done
