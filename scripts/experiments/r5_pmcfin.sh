#!/bin/bash
# PMC passes of the round-5 kernels: headline and reference workload (l0s split)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
timeout -k 10 600 bash scripts/experiments/r4_pmc.sh r5pf_head --steps 20 --warmup 5 || exit $?
timeout -k 10 600 bash scripts/experiments/r4_pmc.sh r5pf_ref --preset reference --embedding_size 32 --batch_size 1024 --steps 64 --warmup 5 || exit $?
ls gpurun_out/r5pf_*
exit 0
