#!/bin/bash
# Timeline of the streamed (uncached) input path: generate Kaggle-shape TFRecords, then the
# data bench's streamed arm under rocprofv3 with kernel + memory-copy traces; summary of the
# copies (H2D bandwidth) and of the kernels per batch.  usage: scripts/stream_prof.sh <tag> <rows>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${1:-sp}; ROWS=${2:-4000000}
export TMPDIR=/tmp
D=/tmp/hipfm_sp_$$
timeout -k 10 600 python tools/gen_synthetic_criteo.py --out "$D" --preset criteo_kaggle \
  --train_rows "$ROWS" --val_rows 16384 --files 16 > gpurun_out/${TAG}_datagen.log 2>&1 || { echo datagen failed; exit 1; }
timeout -k 10 300 python bench.py --data "$D" --preset criteo_kaggle --epochs 3 --stream_only > gpurun_out/${TAG}_plain.log 2>&1; rc=$?
echo "plain rc=$rc: $(tail -1 gpurun_out/${TAG}_plain.log)"
[ $rc -ne 0 ] && { rm -rf "$D"; exit $rc; }
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_$TAG" -o run -- \
  python3 "$ROOT/bench.py" --data "$D" --preset criteo_kaggle --epochs 3 --stream_only > gpurun_out/${TAG}_prof.log 2>&1; rc=$?
echo "prof rc=$rc: $(tail -1 gpurun_out/${TAG}_prof.log)"
rm -rf "$D"
python tools/stream_summary.py "gpurun_out/prof_$TAG" > gpurun_out/${TAG}_stream.md 2>&1
head -40 gpurun_out/${TAG}_stream.md
rm -rf "gpurun_out/prof_$TAG"
exit 0
