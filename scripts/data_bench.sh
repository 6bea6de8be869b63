#!/bin/bash
# File-fed bench: generate Kaggle-shape synthetic TFRecords on the box's local disk, then
# bench.py --data (host ingest rate + Estimator train rate: epoch 0 streamed, later epochs cached).
# usage: scripts/data_bench.sh <rows> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROWS=${1:-1000000}; shift
D=${TMPDIR:-/tmp}/hipfm_data_$$
timeout -k 10 600 python tools/gen_synthetic_criteo.py --out "$D" --preset criteo_kaggle \
  --train_rows "$ROWS" --val_rows 65536 --files 16 > gpurun_out/datagen.log 2>&1 || { echo "datagen failed"; tail -5 gpurun_out/datagen.log; exit 1; }
du -sh "$D"
timeout -k 10 600 python bench.py --data "$D" --preset criteo_kaggle "$@" > gpurun_out/data_bench.log 2>&1
rc=$?; tail -1 gpurun_out/data_bench.log; echo "data bench rc=$rc"
rm -rf "$D"
exit $rc
