#!/bin/bash
# One GPU call: stamp profile + driver-shaped bench + the GPU tests named in $TESTS (pytest -k).
# usage: TESTS="<pytest -k expr>" FILES="tests/a.py tests/b.py" scripts/r4_check.sh <tag> [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=$1; shift
A="${@:---steps 20 --warmup 5}"
bash scripts/experiments/r4_stamps.sh "$TAG" $A || exit $?
timeout -k 10 300 python bench.py $A > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench.log
if [ -n "$FILES" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $FILES ${TESTS:+-k "$TESTS"} \
    > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
  tail -3 gpurun_out/${TAG}_pytest.log
  exit $rc
fi
