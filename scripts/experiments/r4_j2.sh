#!/bin/bash
# PMC passes of the headline config with fp32 and with bf16 embedding records.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r4j}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
bash scripts/experiments/r4_pmc.sh ${TAG}_pmc_fp32 --steps 20 --warmup 5 > gpurun_out/${TAG}_pmc_fp32.log 2>&1; rc=$?; fatal $rc pmc_fp32
bash scripts/experiments/r4_pmc.sh ${TAG}_pmc_bf16 --steps 20 --warmup 5 --emb_dtype bf16 > gpurun_out/${TAG}_pmc_bf16.log 2>&1; rc=$?; fatal $rc pmc_bf16
L=$PWD/deepfm-tensorflow-distributed-training-on-sagemaker_amd/_lib
for v in base nr nd; do
  so=$L/libhipfm_kernels_$v.so; [ $v = base ] && so=$L/libhipfm_kernels.so
  [ -f $so ] || continue
  HIPFM_KERNELS_SO=$so bash scripts/profile.sh "${TAG}_ow_$v" --steps 20 --warmup 5 --force_exchange > /dev/null 2>&1; rc=$?; fatal $rc ow_$v
  python tools/prof_summary.py "gpurun_out/prof_${TAG}_ow_$v" "gpurun_out/${TAG}_ow_${v}_kernels.md" "$TAG owner variant $v" > /dev/null
  rm -rf "gpurun_out/prof_${TAG}_ow_$v"
  echo "owner $v: $(grep -A9 'One steady' gpurun_out/${TAG}_ow_${v}_kernels.md | grep sh_apply_dense)"
done
# packed-FP32 build: determinism tests + A/B bench against the default build
PK=$L/libhipfm_kernels_pk.so
if [ -f $PK ]; then
  HIPFM_KERNELS_SO=$PK timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_determinism.py > gpurun_out/${TAG}_pk_det.log 2>&1; rc=$?
  fatal $rc pk_det
  echo "packed determinism: rc=$rc $(tail -1 gpurun_out/${TAG}_pk_det.log)"
  for k in 1 2; do
    for so in $L/libhipfm_kernels.so $PK; do
      HIPFM_KERNELS_SO=$so timeout -k 10 300 python bench.py --steps 100 --warmup 5 > gpurun_out/${TAG}_pkab.log 2>&1; rc=$?
      fatal $rc pkab
      echo "$(basename $so) run $k: $(tail -1 gpurun_out/${TAG}_pkab.log | grep -o '"ms_per_step": [0-9.]*')"
    done
  done
fi
echo "pmc done"; grep "sfwg_kernel\|tower_kernel" gpurun_out/${TAG}_pmc_*_pmc_raw.md | cut -c1-200
exit 0
