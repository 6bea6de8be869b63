#!/bin/bash
# Streamed input path after the ring fix: the e2e ring test alone first, then the file-fed bench
# (2M rows, the VERDICT's config) and the streamed-path timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r4k}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_e2e.py -k streamed > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
fatal $rc pytest
echo "pytest rc=$rc: $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -ne 0 ] && { grep -E "Error|FAILED" gpurun_out/${TAG}_pytest.log | head -10; exit $rc; }
bash scripts/data_bench.sh 2000000 --epochs 3; rc=$?; fatal $rc data
[ $rc -ne 0 ] && exit $rc
bash scripts/stream_prof.sh ${TAG}s 4000000; rc=$?; fatal $rc stream
exit 0
