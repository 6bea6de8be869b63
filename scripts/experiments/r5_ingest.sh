#!/bin/bash
# host ingest rate vs decode threads / copy threads / per-worker queue depth (16M Kaggle rows)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
D=/tmp/hipfm_ing_$$
timeout -k 10 600 python tools/gen_synthetic_criteo.py --out "$D" --preset criteo_kaggle --train_rows 16000000 \
  --val_rows 16384 --files 64 > gpurun_out/r5i_datagen.log 2>&1 || { echo datagen failed; exit 1; }
timeout -k 10 600 python tools/ingest_sweep.py "$D" 39 16384 2>&1 | tee gpurun_out/r5i_ingest.log
rm -rf "$D"
