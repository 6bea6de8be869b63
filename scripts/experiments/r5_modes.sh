#!/bin/bash
# replicated in-place gradient-row gather + single-wide-layer tower: tests, Kaggle modes, repl profile
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_shard.py::test_replicated_exchange_matches_global_batch tests/test_gpu_shard.py::test_overlapped_exchange_matches_default tests/test_gpu_dist1.py tests/test_gpu_dx0_split.py \
  > gpurun_out/${TAG:-r5m}_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/${TAG:-r5m}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG:-r5m}_tests.log
bash scripts/experiments/r4_modes.sh ${TAG:-r5m} || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG:-r5m}_repl -o run -- \
  python3 bench.py --preset criteo_kaggle --steps 50 --warmup 5 --sparse_update lazy --force_exchange \
  --embedding_mode replicated > gpurun_out/prof_${TAG:-r5m}_repl.log 2>&1 || { echo "prof failed rc=$?"; exit 1; }
[ -n "$SKIP_TF1" ] && { echo profiles done; exit 0; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG:-r5m}_repl_tf1 -o run -- \
  python3 bench.py --preset criteo_kaggle --steps 50 --warmup 5 --sparse_update tf1_dense --force_exchange \
  --embedding_mode replicated > gpurun_out/prof_${TAG:-r5m}_repl_tf1.log 2>&1 || { echo "prof tf1 failed rc=$?"; exit 1; }
echo profiles done
