#!/bin/bash
# Round-end check: the whole GPU suite file by file, smoke(), three driver-shaped headline benches,
# the headline timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r4f}
fatal() { case $1 in 0) ;; 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; *) echo "rc=$1 at $2";; esac; }
bash scripts/r4_n.sh ${TAG}; fatal $? suite
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$?
echo "smoke rc=$rc: $(tail -1 gpurun_out/${TAG}_smoke.log)"; fatal $rc smoke
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench$k.log 2>&1; fatal $? bench
  echo "bench run $k: $(tail -1 gpurun_out/${TAG}_bench$k.log | grep -o '"ms_per_step": [0-9.]*')"
done
timeout -k 10 400 bash scripts/prof_kernels.sh "${TAG}_head|--steps 20 --warmup 5"; fatal $? prof
grep -A8 "One steady-state" gpurun_out/${TAG}_head_kernels.md
exit 0
