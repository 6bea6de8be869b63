#!/bin/bash
# Streamed epochs, GPU decode + GPU data CRC (HIPFM_GPU_DECODE=1), GPU decode + host CRC (2), host
# decode + compact wire (0), interleaved (ARMS="1 2 0" picks the arms):
# Kaggle-shape TFRecords generated on the box, bench.py --data --stream_only per arm.
# usage: scripts/stream_decode_ab.sh <rows> <files> <rounds> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROWS=${1:-16000000}; FILES=${2:-64}; ROUNDS=${3:-2}; shift 3
D=${TMPDIR:-/tmp}/hipfm_stream_$$
timeout -k 10 900 python tools/gen_synthetic_criteo.py --out "$D" --preset criteo_kaggle \
  --train_rows "$ROWS" --val_rows 16384 --files "$FILES" > gpurun_out/stream_datagen.log 2>&1 || { echo "datagen failed"; tail -5 gpurun_out/stream_datagen.log; exit 1; }
du -sh "$D"
for r in $(seq 1 "$ROUNDS"); do
  for g in ${ARMS:-1 0}; do
    HIPFM_GPU_DECODE=$g timeout -k 10 300 python bench.py --data "$D" --preset criteo_kaggle --stream_only "$@" \
      > gpurun_out/stream_ab_g${g}_r$r.log 2>&1 || { echo "arm g=$g failed"; tail -5 gpurun_out/stream_ab_g${g}_r$r.log; rm -rf "$D"; exit 1; }
    echo "gpu_decode=$g run=$r $(tail -1 gpurun_out/stream_ab_g${g}_r$r.log | cut -c1-400)"
  done
done
rm -rf "$D"
