#!/bin/bash
# PMC passes over streamed epochs with the GPU Example decoder (decode_examples_kernel + CRC):
# Kaggle-shape TFRecords generated on the box, bench.py --data --stream_only, two counter passes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
D=${TMPDIR:-/tmp}/hipfm_dpmc_$$
timeout -k 10 600 python tools/gen_synthetic_criteo.py --out "$D" --preset criteo_kaggle --train_rows 4000000 \
  --val_rows 16384 --files 16 > gpurun_out/dpmc_datagen.log 2>&1 || { echo "datagen failed"; rm -rf "$D"; exit 1; }
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="FETCH_SIZE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_COUNT"
rc=0
bash scripts/pmc.sh dec1 "$P1" --data "$D" --preset criteo_kaggle --stream_only --epochs 2 > gpurun_out/dpmc1.txt 2>&1 || rc=1
[ $rc -eq 0 ] && { bash scripts/pmc.sh dec2 "$P2" --data "$D" --preset criteo_kaggle --stream_only --epochs 2 > gpurun_out/dpmc2.txt 2>&1 || rc=1; }
rm -rf "$D"
[ $rc -ne 0 ] && { cat gpurun_out/dpmc1.txt gpurun_out/dpmc2.txt; exit 1; }
python tools/pmc_raw.py gpurun_out/r6_decode_pmc_raw.md "r6: streamed epochs, GPU decode + CRC (bench --stream_only, 4M rows)" gpurun_out/pmc_dec1 gpurun_out/pmc_dec2
rm -rf gpurun_out/pmc_dec1 gpurun_out/pmc_dec2
