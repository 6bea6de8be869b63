#!/bin/bash
# bf16 embeddings vs fp32 (PMC of both at the headline config), the K = 32 Criteo-1TB table with
# bf16 records on one GPU, and the Kaggle replicated proxy's kernel timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r4j}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_plan_state.py tests/test_gpu_determinism.py > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
fatal $rc pytest
echo "pytest rc=$rc: $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -ne 0 ] && grep -E "Error|FAILED|invariant" gpurun_out/${TAG}_pytest.log | head -10
for e in fp32 bf16; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --emb_dtype $e > gpurun_out/${TAG}_emb_$e.log 2>&1; rc=$?
  fatal $rc emb_$e
  echo "emb $e: $(tail -1 gpurun_out/${TAG}_emb_$e.log | grep -o '"ms_per_step": [0-9.]*'), auc $(tail -1 gpurun_out/${TAG}_emb_$e.log | grep -o '"eval_auc": [0-9.]*')"
done
timeout -k 10 900 python bench.py --steps 20 --warmup 5 --embedding_size 32 --emb_dtype bf16 > gpurun_out/${TAG}_k32_bf16.log 2>&1; rc=$?
fatal $rc k32
echo "k32 bf16 1TB: rc=$rc $(tail -1 gpurun_out/${TAG}_k32_bf16.log | cut -c1-600)"
bash scripts/profile.sh "${TAG}_repl" --preset criteo_kaggle --steps 50 --warmup 5 --force_exchange --embedding_mode replicated > /dev/null 2>&1; rc=$?; fatal $rc repl
python tools/prof_summary.py "gpurun_out/prof_${TAG}_repl" "gpurun_out/${TAG}_repl_kernels.md" "$TAG: Kaggle replicated proxy" > /dev/null
rm -rf "gpurun_out/prof_${TAG}_repl"
grep -A14 "One steady-state" gpurun_out/${TAG}_repl_kernels.md
bash scripts/experiments/r4_stamps.sh ${TAG}_ref --preset reference --embedding_size 32 --batch_size 1024 --steps 50 --warmup 5; rc=$?; fatal $rc ref_stamps
bash scripts/pk_bisect.sh 300; rc=$?; fatal $rc pk
exit 0
