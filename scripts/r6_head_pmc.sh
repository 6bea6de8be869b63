#!/bin/bash
# Final headline PMC: 4 counter passes over bench --steps 20 --warmup 5, one table
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"
P3="FETCH_SIZE"
P4="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
i=0
for C in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  bash scripts/pmc.sh r6head_p$i "$C" --steps 20 --warmup 5 > gpurun_out/r6head_p$i.txt 2>&1 || { cat gpurun_out/r6head_p$i.txt; exit 1; }
done
python tools/pmc_raw.py gpurun_out/r6_head_pmc_raw.md "r6 headline PMC: bench --steps 20 --warmup 5" \
  gpurun_out/pmc_r6head_p1 gpurun_out/pmc_r6head_p2 gpurun_out/pmc_r6head_p3 gpurun_out/pmc_r6head_p4
rm -rf gpurun_out/pmc_r6head_p*
