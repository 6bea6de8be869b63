#!/bin/bash
# pinned buffers handed back after their copy (not after the expand kernel): streamed-ring test,
# then streamed epochs (16M Kaggle rows), compact 1 / 0, x2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_e2e.py::test_streamed_epochs_through_the_ring_train_like_the_cached_run \
  > gpurun_out/r5e_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r5e_tests.log; exit 1; }
tail -1 gpurun_out/r5e_tests.log
D=/tmp/hipfm_ev_$$
timeout -k 10 600 python tools/gen_synthetic_criteo.py --out "$D" --preset criteo_kaggle --train_rows 16000000 \
  --val_rows 16384 --files 64 > gpurun_out/r5e_datagen.log 2>&1 || { echo datagen failed; exit 1; }
for r in 1 2; do
  for c in 1 0; do
    HIPFM_WIRE_COMPACT=$c timeout -k 10 300 python bench.py --data "$D" --preset criteo_kaggle --epochs 3 \
      --stream_only --threads 16 > gpurun_out/r5e_c${c}_$r.log 2>&1 || { echo "bench c=$c failed"; rm -rf "$D"; exit 1; }
    echo "compact=$c run=$r $(tail -1 gpurun_out/r5e_c${c}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["streamed_epoch_samples_per_s"], d["fill_thread_last_epoch"], d["epoch_s"])')"
  done
done
rm -rf "$D"
