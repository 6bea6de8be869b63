#!/bin/bash
# Kernel trace + occupancy / stall / memory PMC passes of one bench configuration, summarised on
# the box (gpurun_out/<tag>_kernels.md, <tag>_pmc_raw.md).  One pass per counter group (rocprofv3
# does not split counters over passes); a pass that times out or crashes ends the script.
# usage: scripts/experiments/r4_pmc.sh <tag> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
TAG=$1; shift
A="${@:---steps 20 --warmup 5}"
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
bash scripts/profile.sh "$TAG" $A; rc=$?
if fatal $rc; then echo "trace pass rc=$rc: stop"; exit $rc; fi
python tools/prof_summary.py "gpurun_out/prof_$TAG" "gpurun_out/${TAG}_kernels.md" "$TAG: bench $A"
rm -rf "gpurun_out/prof_$TAG"
dirs=()
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
            "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum"; do
  i=$((i + 1))
  bash scripts/pmc.sh "${TAG}_p$i" "$ctrs" $A; rc=$?
  if fatal $rc; then echo "pmc pass $i rc=$rc: stop"; break; fi
  dirs+=("gpurun_out/pmc_${TAG}_p$i")
done
python tools/pmc_raw.py "gpurun_out/${TAG}_pmc_raw.md" "$TAG PMC: bench $A" "${dirs[@]}"
rm -rf "${dirs[@]}"
