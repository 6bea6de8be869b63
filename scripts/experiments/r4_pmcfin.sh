#!/bin/bash
# PMC passes of the final kernels: headline and reference workload
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
timeout -k 10 600 bash scripts/experiments/r4_pmc.sh r4pf_head --steps 20 --warmup 5 || exit $?
timeout -k 10 600 bash scripts/experiments/r4_pmc.sh r4pf_ref --preset reference --embedding_size 32 --batch_size 1024 --steps 64 --warmup 5 || exit $?
ls gpurun_out/r4pf_*
exit 0
