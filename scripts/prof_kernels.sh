#!/bin/bash
# Kernel-trace timelines of several bench configurations in one GPU call, summarised on the box
# (gpurun_out/<tag>_kernels.md).  usage: scripts/prof_kernels.sh "<tag>|<bench args>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for spec in "$@"; do
  TAG="${spec%%|*}"; A="${spec#*|}"
  bash scripts/profile.sh "$TAG" $A || exit $?
  python tools/prof_summary.py "gpurun_out/prof_$TAG" "gpurun_out/${TAG}_kernels.md" "$TAG: bench $A" || exit $?
  rm -rf "gpurun_out/prof_$TAG"
done
