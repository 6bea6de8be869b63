#!/bin/bash
# One GPU call: new GPU tests, Kaggle mode sweep, PMC of the sharded proxy, streamed-path timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r4g}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dist1.py tests/test_gpu_tf1.py > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
fatal $rc pytest
echo "pytest rc=$rc: $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -ne 0 ] && exit $rc
bash scripts/experiments/r4_modes.sh ${TAG}m; rc=$?; fatal $rc modes
bash scripts/experiments/r4_pmc.sh ${TAG}_pxpmc --steps 20 --warmup 5 --force_exchange > gpurun_out/${TAG}_pmc.log 2>&1; rc=$?; fatal $rc pmc
echo "pmc rc=$rc"
bash scripts/stream_prof.sh ${TAG}s 4000000; rc=$?; fatal $rc stream
exit 0
