#!/bin/bash
# streamed epochs vs loader threads (Kaggle shape, 4M rows, 16 files)
cd $GRAFT_REPO_ROOT
D=/tmp/hipfm_st_$$
timeout -k 10 600 python tools/gen_synthetic_criteo.py --out "$D" --preset criteo_kaggle --train_rows 4000000 \
  --val_rows 16384 --files 32 > gpurun_out/r5w_datagen.log 2>&1 || { echo datagen failed; exit 1; }
nproc; python -c "import os; print(len(os.sched_getaffinity(0)))"
for t in 8 12 16 24; do
  timeout -k 10 300 python bench.py --data "$D" --preset criteo_kaggle --epochs 3 --stream_only --threads $t > gpurun_out/r5w_t$t.log 2>&1
  echo "threads=$t rc=$? $(tail -1 gpurun_out/r5w_t$t.log | cut -c1-260)"
done
rm -rf "$D"
