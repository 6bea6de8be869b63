#!/bin/bash
# Streamed epochs with GPU decode at several loader thread counts (one dataset, generated once).
# usage: scripts/stream_threads.sh <rows> <files> "<thread counts>" [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROWS=${1:-16000000}; FILES=${2:-64}; TH=${3:-"8 16"}; shift 3
D=${TMPDIR:-/tmp}/hipfm_stream_$$
timeout -k 10 900 python tools/gen_synthetic_criteo.py --out "$D" --preset criteo_kaggle \
  --train_rows "$ROWS" --val_rows 16384 --files "$FILES" > gpurun_out/stream_datagen.log 2>&1 || { echo "datagen failed"; exit 1; }
for t in $TH; do
  for g in ${ARMS:-1 0}; do
    HIPFM_GPU_DECODE=$g timeout -k 10 300 python bench.py --data "$D" --preset criteo_kaggle --stream_only --threads $t "$@" \
      > gpurun_out/stream_t${t}_g$g.log 2>&1 || { echo "t=$t failed"; tail -3 gpurun_out/stream_t${t}_g$g.log; rm -rf "$D"; exit 1; }
    echo "threads=$t gpu_decode=$g $(tail -1 gpurun_out/stream_t${t}_g$g.log | cut -c1-330)"
  done
done
rm -rf "$D"
