cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
run() { echo "== $*"; timeout -k 10 300 env "$@" > gpurun_out/diag_last.log 2>&1; rc=$?; tail -4 gpurun_out/diag_last.log; return $rc; }
run DIAG_PREFETCH=1 python tools/diag/shard_emul_check.py 8 16384 criteo_1tb 2 &&
run DIAG_PREFETCH=0 python tools/diag/shard_emul_check.py 8 16384 criteo_1tb 2 &&
run DIAG_PREFETCH=1 python tools/diag/shard_emul_check.py 8 2048 criteo_1tb 2
