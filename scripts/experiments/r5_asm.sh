#!/bin/bash
# C++ assembly ring (HIPFM_ASM_RING 1 / 0), compact wire format, long epochs (16M rows)
# interleaved x2, after the streamed-vs-cached GPU test
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_e2e.py::test_streamed_epochs_through_the_ring_train_like_the_cached_run \
  > gpurun_out/r5a_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r5a_tests.log; exit 1; }
tail -1 gpurun_out/r5a_tests.log
D=/tmp/hipfm_wx_$$
time timeout -k 10 600 python tools/gen_synthetic_criteo.py --out "$D" --preset criteo_kaggle --train_rows 16000000 \
  --val_rows 16384 --files 64 > gpurun_out/r5a_datagen.log 2>&1 || { echo datagen failed; exit 1; }
du -sh $D
for r in 1 2; do
  for c in 1 0; do
    HIPFM_ASM_RING=$c timeout -k 10 300 python bench.py --data "$D" --preset criteo_kaggle --epochs 3 \
      --stream_only --threads 16 > gpurun_out/r5a_c${c}_$r.log 2>&1 || { echo "bench c=$c failed"; tail -5 gpurun_out/r5a_c${c}_$r.log; rm -rf "$D"; exit 1; }
    echo "asm=$c run=$r $(tail -1 gpurun_out/r5a_c${c}_$r.log | cut -c1-330)"
  done
done
rm -rf "$D"
