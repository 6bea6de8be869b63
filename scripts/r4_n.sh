#!/bin/bash
# Full GPU test suite, verbose, one file at a time (a stalled test names itself).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r4n}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
for f in tests/test_gpu_*.py; do
  echo "== $f" >> gpurun_out/${TAG}_pytest.log
  timeout -k 10 400 python -u -m pytest -v --timeout 150 --timeout-method thread $f >> gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
  echo "$f rc=$rc: $(tail -1 gpurun_out/${TAG}_pytest.log)"
  fatal $rc $f
done
exit 0
