cd "${GRAFT_REPO_ROOT}"
A="--preset criteo_kaggle --sparse_update tf1_dense --steps 100 --warmup 10"
bash scripts/pmc.sh tf1f "FETCH_SIZE GRBM_GUI_ACTIVE" $A || exit $?
bash scripts/pmc.sh tf1w "WRITE_SIZE" $A || exit $?
bash scripts/pmc.sh tf1s "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" $A || exit $?
