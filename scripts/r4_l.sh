#!/bin/bash
# Replicated run-level routing (tests + Kaggle mode sweep) and the streamed path with two copy streams.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r4l}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dist1.py tests/test_gpu_shard.py tests/test_gpu_e2e.py -k "replicated or streamed or run_routing or tf1_split" > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
fatal $rc pytest
echo "pytest rc=$rc: $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -ne 0 ] && { grep -E "Error|FAILED" gpurun_out/${TAG}_pytest.log | head -10; exit $rc; }
bash scripts/r4_modes.sh ${TAG}m; rc=$?; fatal $rc modes
bash scripts/stream_prof.sh ${TAG}s 4000000; rc=$?; fatal $rc stream
exit 0
