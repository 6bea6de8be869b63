cd "${GRAFT_REPO_ROOT}"
bash scripts/profile.sh r2qfx --force_exchange --steps 100 --warmup 10 || exit $?
python tools/prof_summary.py gpurun_out/prof_r2qfx gpurun_out/r2q_fx_kernels.md "r2q: row-sharded step on a 1-rank RCCL group (--force_exchange)" || exit $?
rm -rf gpurun_out/prof_r2qfx
bash scripts/profile.sh r2qt --preset criteo_kaggle --sparse_update tf1_dense --steps 100 --warmup 10 || exit $?
python tools/prof_summary.py gpurun_out/prof_r2qt gpurun_out/r2q_tf1_merged_kernels.md "r2q: Kaggle-shape tf1_dense, merged sweep (sweep workgroups inside the sparse + wgfin launch)" || exit $?
rm -rf gpurun_out/prof_r2qt
