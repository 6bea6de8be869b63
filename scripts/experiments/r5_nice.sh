#!/bin/bash
# streamed epochs vs the decode workers' nice increment (HIPFM_DECODE_NICE 0 / 5 / 10, a knob since removed: no reproducible effect), 16M rows
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
D=/tmp/hipfm_nice_$$
timeout -k 10 600 python tools/gen_synthetic_criteo.py --out "$D" --preset criteo_kaggle --train_rows 16000000 \
  --val_rows 16384 --files 64 > gpurun_out/r5n_datagen.log 2>&1 || { echo datagen failed; exit 1; }
F0=$(ls $D/tr-*.tfrecords | head -1)
for i in 1 2 3; do
  echo "decode old: $(tools/iobench/decode_old $F0 | tail -1)"
  echo "decode new: $(tools/iobench/decode_new $F0 | tail -1)"
done
for r in 1 2; do
  for n in 0 5 10; do
    HIPFM_DECODE_NICE=$n timeout -k 10 300 python bench.py --data "$D" --preset criteo_kaggle --epochs 3 \
      --stream_only --threads 16 > gpurun_out/r5nice_${n}_$r.log 2>&1 || { echo "bench nice=$n failed"; tail -5 gpurun_out/r5nice_${n}_$r.log; rm -rf "$D"; exit 1; }
    echo "nice=$n run=$r $(tail -1 gpurun_out/r5nice_${n}_$r.log | cut -c1-250)"
  done
done
rm -rf "$D"
