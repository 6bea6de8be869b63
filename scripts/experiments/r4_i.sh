#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r4i}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_e2e.py tests/test_gpu_dist1.py tests/test_gpu_shard.py > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
fatal $rc pytest
echo "pytest rc=$rc: $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -ne 0 ] && grep -E "Error|FAILED" gpurun_out/${TAG}_pytest.log | head -10
for site in sfwg tower sfwg tower; do
  HIPFM_SERVE_SITE=$site timeout -k 10 300 python bench.py --steps 20 --warmup 5 --force_exchange > gpurun_out/${TAG}_px_$site.log 2>&1; rc=$?
  fatal $rc px_$site
  echo "px $site: $(tail -1 gpurun_out/${TAG}_px_$site.log | cut -c1-330 | grep -o '"ms_per_step": [0-9.]*')"
done
bash scripts/profile.sh "${TAG}_px" --steps 20 --warmup 5 --force_exchange > /dev/null 2>&1; rc=$?; fatal $rc trace
python tools/prof_summary.py "gpurun_out/prof_${TAG}_px" "gpurun_out/${TAG}_px_kernels.md" "$TAG: bench --force_exchange" > /dev/null
rm -rf "gpurun_out/prof_${TAG}_px"
grep -A12 "One steady-state" gpurun_out/${TAG}_px_kernels.md
bash scripts/io_probe.sh; rc=$?; fatal $rc io
bash scripts/stream_prof.sh ${TAG}s 4000000; rc=$?; fatal $rc stream
bash scripts/data_bench.sh 2000000 --epochs 3; rc=$?; fatal $rc data
exit 0
