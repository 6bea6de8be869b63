#!/bin/bash
# wgfin head reduction over > 256 columns (last deep layer 256): diagnostic + tests + modes + repl profile
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python tools/diag/r5_nl1_grads.py > gpurun_out/r5_nl1b.log 2>&1 || { echo diag failed; tail -5 gpurun_out/r5_nl1b.log; exit 1; }
grep -E "^\[|fm_bias|deep_out/biases" gpurun_out/r5_nl1b.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_dx0_split.py tests/test_gpu_kernels.py \
  > gpurun_out/r5n_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r5n_tests.log; exit 1; }
tail -1 gpurun_out/r5n_tests.log
bash scripts/experiments/r5_modes.sh
