#!/bin/bash
# PMC passes (counters only with --kernel-trace/--stats) of one wide-layer GEMM (tools/gemm_one.py).
# usage: scripts/gemm_pmc.sh <tag> [gemm_one args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=$1; shift
export TMPDIR=/tmp
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_COUNT"
i=0
for CTRS in "$P1" "$P2"; do
  i=$((i+1))
  mkdir -p gpurun_out/gpmc_${TAG}_$i
  timeout -s KILL 90 rocprofv3 --pmc $CTRS --kernel-trace --stats --output-format csv \
    -d "$ROOT/gpurun_out/gpmc_${TAG}_$i" -o run -- python3 "$ROOT/tools/gemm_one.py" "$@" \
    > "$ROOT/gpurun_out/gpmc_${TAG}_$i/log.txt" 2>&1 || { echo "pass $i failed"; tail -5 "$ROOT/gpurun_out/gpmc_${TAG}_$i/log.txt"; exit 1; }
done
echo ok
