#!/bin/bash
# Phase stamps of the tower / sparse launches (diagnostic stamp library, built on the CPU with
# HIPFM_BUILD_STAMPS=1) for one bench configuration: gpurun_out/<tag>_stamps.md
# usage: scripts/experiments/r4_stamps.sh <tag> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=$1; shift
A="${@:---steps 20 --warmup 5}"
LIB=$(pwd)/deepfm-tensorflow-distributed-training-on-sagemaker_amd/_lib/libhipfm_kernels_stamps.so
HIPFM_KERNELS_SO=$LIB HIPFM_BENCH_STAMPS=gpurun_out/${TAG}_stamps.npz timeout -k 10 300 \
  python bench.py $A > gpurun_out/${TAG}_stamps.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_stamps.log
python tools/stamps.py gpurun_out/${TAG}_stamps.npz gpurun_out/${TAG}_stamps.md > /dev/null
