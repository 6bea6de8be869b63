cd "${GRAFT_REPO_ROOT}"
A="--steps 100 --warmup 10"
bash scripts/profile.sh r2q $A || exit $?
bash scripts/pmc.sh r2qf "FETCH_SIZE GRBM_GUI_ACTIVE" $A || exit $?
bash scripts/pmc.sh r2qw "WRITE_SIZE" $A || exit $?
bash scripts/pmc.sh r2qs "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" $A || exit $?
