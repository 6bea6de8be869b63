#!/bin/bash
# Quick check of a kernel change: the given GPU test files (one pytest process), then the 1-GPU
# bench line N times.  usage: scripts/quick_ab.sh TAG NBENCH "test files" [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=$1; NB=$2; TESTS=$3; shift 3
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q -m gpu --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -1 gpurun_out/${TAG}_pytest.log)"
  [ $rc -eq 0 ] || exit $rc
fi
for i in $(seq 1 $NB); do
  timeout -k 10 300 python bench.py "$@" > gpurun_out/${TAG}_bench_$i.log 2>&1
  rc=$?; echo "bench[$i] rc=$rc: $(tail -1 gpurun_out/${TAG}_bench_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("eval_auc"))' 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
done
