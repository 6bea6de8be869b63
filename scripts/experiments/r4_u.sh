#!/bin/bash
# Reference workload: the FM gather in the tower's prologue (default) vs an fm_fwd launch across
# the chip (HIPFM_TOWER_GATHER=0), lazy and tf1_dense; timeline of the unfused step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r4u}
fatal() { case $1 in 0) ;; 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; *) echo "rc=$1 at $2"; exit $1;; esac; }
R="--preset reference --embedding_size 32 --batch_size 1024 --steps 100 --warmup 5"
for k in 1 2; do
  for g in 1 0; do
    HIPFM_TOWER_GATHER=$g timeout -k 10 300 python bench.py $R > gpurun_out/${TAG}_ref_g$g.log 2>&1; fatal $? ref_g$g
    echo "ref lazy gather=$g run $k: $(tail -1 gpurun_out/${TAG}_ref_g$g.log | grep -o '"ms_per_step": [0-9.]*')"
    HIPFM_TOWER_GATHER=$g timeout -k 10 300 python bench.py $R --sparse_update tf1_dense > gpurun_out/${TAG}_ref_tf1_g$g.log 2>&1; fatal $? ref_tf1_g$g
    echo "ref tf1 gather=$g run $k: $(tail -1 gpurun_out/${TAG}_ref_tf1_g$g.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
HIPFM_TOWER_GATHER=0 timeout -k 10 400 bash scripts/prof_kernels.sh "${TAG}_ref_g0|--preset reference --embedding_size 32 --batch_size 1024 --steps 64 --warmup 5"; fatal $? prof
grep -A10 "One steady-state" gpurun_out/${TAG}_ref_g0_kernels.md
exit 0
