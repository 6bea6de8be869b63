#!/bin/bash
# Kernel trace + three PMC passes of a bench run, summarised ON the box (the raw CSVs exceed
# gpurun's 64 MiB copy-back): gpurun_out/<tag>_kernels.md and <tag>_pmc.md.
# usage: scripts/r2q_prof.sh <tag> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r2q}; shift
A="${@:---steps 100 --warmup 10}"
bash scripts/profile.sh "$TAG" $A || exit $?
python tools/prof_summary.py "gpurun_out/prof_$TAG" "gpurun_out/${TAG}_kernels.md" "$TAG: bench $A" || exit $?
rm -rf "gpurun_out/prof_$TAG"
bash scripts/pmc.sh "${TAG}f" "FETCH_SIZE GRBM_GUI_ACTIVE" $A || exit $?
bash scripts/pmc.sh "${TAG}w" "WRITE_SIZE" $A || exit $?
bash scripts/pmc.sh "${TAG}s" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" $A || exit $?
python tools/pmc_summary.py "gpurun_out/${TAG}_pmc.md" "$TAG PMC counters: bench $A" \
  "gpurun_out/pmc_${TAG}f" "gpurun_out/pmc_${TAG}w" "gpurun_out/pmc_${TAG}s" || exit $?
rm -rf "gpurun_out/pmc_${TAG}f" "gpurun_out/pmc_${TAG}w" "gpurun_out/pmc_${TAG}s"
