#!/bin/bash
# round 6: the box's file-read bandwidth over a streamed dataset (the streamed-epoch ceiling), then
# the full one-process GPU suite and the smoke
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
D=${TMPDIR:-/tmp}/hipfm_rbw_$$
df -h "${TMPDIR:-/tmp}" > gpurun_out/rbw_df.txt 2>&1
timeout -k 10 600 python tools/gen_synthetic_criteo.py --out "$D" --preset criteo_kaggle --train_rows 16000000 \
  --val_rows 16384 --files 64 > gpurun_out/rbw_datagen.log 2>&1 || { echo "datagen failed"; rm -rf "$D"; exit 1; }
timeout -k 10 300 python tools/read_bw.py "$D" --threads 1,4,8,16 --passes 2 > gpurun_out/rbw.json 2>&1; rc=$?
rm -rf "$D"; cat gpurun_out/rbw.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_suite.log 2>&1
rc=$?; tail -2 gpurun_out/r6_suite.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/r6_smoke.log; exit $rc
