#!/bin/bash
# PMC passes of the headline config with fp32 and with bf16 embedding records.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r4j}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
bash scripts/r4_pmc.sh ${TAG}_pmc_fp32 --steps 20 --warmup 5 > gpurun_out/${TAG}_pmc_fp32.log 2>&1; rc=$?; fatal $rc pmc_fp32
bash scripts/r4_pmc.sh ${TAG}_pmc_bf16 --steps 20 --warmup 5 --emb_dtype bf16 > gpurun_out/${TAG}_pmc_bf16.log 2>&1; rc=$?; fatal $rc pmc_bf16
echo "pmc done"; grep "sfwg_kernel\|tower_kernel" gpurun_out/${TAG}_pmc_*_pmc_raw.md | cut -c1-200
exit 0
