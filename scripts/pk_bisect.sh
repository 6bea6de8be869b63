#!/bin/bash
# Packed-FP32 hazard bisection (tools/pkhazard/bisect.py) over the default and packed builds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$PWD/deepfm-tensorflow-distributed-training-on-sagemaker_amd/_lib
for so in libhipfm_kernels.so libhipfm_kernels_pk.so libhipfm_kernels_pk1.so libhipfm_kernels_pk2.so; do
  [ -f $L/$so ] || continue
  HIPFM_KERNELS_SO=$L/$so timeout -k 10 180 python tools/pkhazard/bisect.py ${1:-300}; rc=$?
  case $rc in 124|134|137|139) echo "fatal rc=$rc at $so"; exit $rc;; esac
done
exit 0
