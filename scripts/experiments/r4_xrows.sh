#!/bin/bash
# Exchange-row formats on the 1-rank sharded proxy: GPU exchange tests, then the proxy bench with
# bf16 and fp32 rows and a kernel trace of the default.  usage: scripts/r4_xrows.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-xr}
export PYTHONPATH=$PWD
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dist1.py tests/test_gpu_shard.py tests/test_gpu_plan_state.py > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
fatal $rc pytest
echo "pytest rc=$rc: $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -ne 0 ] && exit $rc
for xr in bf16 fp32; do
  HIPFM_XROWS=$xr timeout -k 10 300 python bench.py --steps 20 --warmup 5 --force_exchange > gpurun_out/${TAG}_px_$xr.log 2>&1; rc=$?
  fatal $rc px_$xr
  echo "px $xr rc=$rc: $(tail -1 gpurun_out/${TAG}_px_$xr.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["eval_auc"], d.get("comm_bytes_moved_per_step"))')"
done
bash scripts/profile.sh "${TAG}_px" --steps 20 --warmup 5 --force_exchange > /dev/null 2>&1; rc=$?; fatal $rc proxy_trace
python tools/prof_summary.py "gpurun_out/prof_${TAG}_px" "gpurun_out/${TAG}_px_kernels.md" "$TAG: bench --force_exchange" > /dev/null
rm -rf "gpurun_out/prof_${TAG}_px"
# owner-update diagnostic variants (wrong results, timing only): no probe / no patch / neither
for v in np nq nb; do
  so=$PWD/deepfm-tensorflow-distributed-training-on-sagemaker_amd/_lib/libhipfm_kernels_$v.so
  [ -f $so ] || continue
  HIPFM_KERNELS_SO=$so bash scripts/profile.sh "${TAG}_$v" --steps 20 --warmup 5 --force_exchange > /dev/null 2>&1; rc=$?; fatal $rc trace_$v
  python tools/prof_summary.py "gpurun_out/prof_${TAG}_$v" "gpurun_out/${TAG}_${v}_kernels.md" "$TAG variant $v" > /dev/null
  rm -rf "gpurun_out/prof_${TAG}_$v"
  echo "variant $v: $(grep -m1 sh_apply_dense gpurun_out/${TAG}_${v}_kernels.md)"
done
exit 0
