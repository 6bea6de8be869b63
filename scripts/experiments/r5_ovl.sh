#!/bin/bash
# overlap mode: GPU tests, then the 1-rank proxy with and without it
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_dist1.py -x -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5r_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 gpurun_out/r5r_pytest.log)"; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r5r_pytest.log | head -20; exit $rc; }
for i in 1 2; do
  for o in 0 1; do
    HIPFM_SH_OVERLAP=$o timeout -k 10 300 python bench.py --steps 20 --warmup 5 --force_exchange > gpurun_out/r5r_px_$o_$i.log 2>&1
    echo "overlap=$o $(tail -1 gpurun_out/r5r_px_$o_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["exec"], d["config"].get("exchange_overlap"))' 2>&1 | tail -1)"
  done
done
