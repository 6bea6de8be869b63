#!/bin/bash
# same-box A/B of the headline: the tree at oldtree_ab (an older commit, built) vs this tree
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  (cd oldtree_ab && timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/ab_old_$i.log 2>&1)
  echo "old $(tail -1 gpurun_out/ab_old_$i.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])' 2>&1 | tail -1)"
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_new_$i.log 2>&1
  echo "new $(tail -1 gpurun_out/ab_new_$i.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])' 2>&1 | tail -1)"
done
