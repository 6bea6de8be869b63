#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (no PMC here; counters go in their own run).
# usage: scripts/profile.sh <tag> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_$TAG" -o run -- \
  python3 "$ROOT/bench.py" "$@" > "$ROOT/gpurun_out/prof_$TAG/bench.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 "$ROOT/gpurun_out/prof_$TAG/bench.log"
find "$ROOT/gpurun_out/prof_$TAG" -name "*kernel_stats.csv" | head -3
exit $rc
