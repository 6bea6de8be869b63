#!/bin/bash
# replicated lazy proxy vs the local step, alternating on one box (Kaggle shape), after the tests
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r5w}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_shard.py::test_replicated_exchange_matches_global_batch tests/test_gpu_dist1.py tests/test_gpu_tf1.py \
  > gpurun_out/${T}_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for i in 1 2 3; do
  for mode in local repl; do
    extra=""; [ $mode = repl ] && extra="--force_exchange --embedding_mode replicated"
    timeout -k 10 300 python bench.py --preset criteo_kaggle --steps 50 --warmup 5 --sparse_update ${UPD:-lazy} $extra \
      > gpurun_out/${T}_${mode}_$i.log 2>&1 || { echo "$mode failed"; tail -5 gpurun_out/${T}_${mode}_$i.log; exit 1; }
    echo "$mode run=$i $(tail -1 gpurun_out/${T}_${mode}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["parallelism"], d["eval_auc"])')"
  done
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_${T}_repl -o run -- \
  python3 bench.py --preset criteo_kaggle --steps 50 --warmup 5 --sparse_update ${UPD:-lazy} --force_exchange \
  --embedding_mode replicated > gpurun_out/prof_${T}_repl.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
