#!/bin/bash
# One rocprofv3 PMC pass (counters only with --kernel-trace/--stats) of a short bench run.
# usage: scripts/pmc.sh <tag> "<counters>" [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=$1; shift
CTRS=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_$TAG
timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-trace --stats --output-format csv \
  -d "$ROOT/gpurun_out/pmc_$TAG" -o run -- python3 "$ROOT/bench.py" "$@" > "$ROOT/gpurun_out/pmc_$TAG/bench.log" 2>&1
rc=$?; echo "pmc rc=$rc"; tail -1 "$ROOT/gpurun_out/pmc_$TAG/bench.log"
exit $rc
