cd "${GRAFT_REPO_ROOT}"
bash scripts/gpu_round.sh "--steps 300 --warmup 50" "--steps 300 --warmup 50 --preset criteo_kaggle --sparse_update tf1_dense" || exit $?
bash scripts/data_bench.sh 2000000 --epochs 5
