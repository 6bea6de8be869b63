#!/bin/bash
# The reference user's flow through the CLI on one GPU, timed per phase: Kaggle-shape TFRecords
# (tr*/va*/te*), train N epochs (epoch 0 streamed + cached, later epochs graph replays), eval,
# infer (pred.txt), export (saved_model.pb + variables).  usage: scripts/cli_e2e.sh <rows> [flags]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROWS=${1:-1000000}; shift
D=${TMPDIR:-/tmp}/hipfm_cli_$$
timeout -k 10 600 python tools/gen_synthetic_criteo.py --out "$D/data" --preset criteo_kaggle \
  --train_rows "$ROWS" --val_rows 65536 --test_rows 65536 --files 8 > gpurun_out/cli_datagen.log 2>&1 || { tail -5 gpurun_out/cli_datagen.log; exit 1; }
FS=$(python -c "from hipfm.data.synthetic import make_synth; print(make_synth('criteo_kaggle').feature_size)")
COMMON="--training_data_dir $D/data --val_data_dir $D/data --model_dir $D/ckpt --servable_model_dir $D/export \
  --feature_size $FS --field_size 39 --embedding_size 8 --batch_size 16384 --deep_layers 128,64,32 \
  --dropout 0.5,0.5,0.5 --optimizer Adam --learning_rate 0.0005 --log_steps 50 $@"
for task in train eval infer export; do
  t0=$(date +%s.%N)
  timeout -k 10 600 python -m hipfm --task_type $task $COMMON > gpurun_out/cli_$task.log 2>&1
  rc=$?; t1=$(date +%s.%N)
  echo "task=$task rc=$rc wall_s=$(python -c "print(round($t1-$t0,1))")"; grep -E "auc|global_step/sec|examples/sec" gpurun_out/cli_$task.log | tail -3
  [ $rc -ne 0 ] && { tail -20 gpurun_out/cli_$task.log; exit $rc; }
done
ls -la "$D/export"/* | head; wc -l "$D"/data/pred.txt 2>/dev/null || find "$D" -name pred.txt -exec wc -l {} \;
rm -rf "$D"
