#!/bin/bash
# Timelines after the counter-rank sort + dX0 split: kernel traces and phase stamps of the headline
# and the reference workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r4s}
fatal() { case $1 in 0) ;; 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; *) echo "rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 400 bash scripts/prof_kernels.sh "${TAG}_head|--steps 20 --warmup 5" "${TAG}_ref|--preset reference --embedding_size 32 --batch_size 1024 --steps 64 --warmup 5"; fatal $? prof
timeout -k 10 300 bash scripts/experiments/r4_stamps.sh ${TAG}_ref --preset reference --embedding_size 32 --batch_size 1024 --steps 64 --warmup 5; fatal $? stamps_ref
timeout -k 10 300 bash scripts/experiments/r4_stamps.sh ${TAG}_head --steps 20 --warmup 5; fatal $? stamps_head
exit 0
