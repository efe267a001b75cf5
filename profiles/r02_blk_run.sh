#!/bin/bash
# Work-block size (GI_X_BLK_LOG2: 64 >> n list entries per block) on the C3 shares and C4
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "mode_x or handoff or shard" > gpurun_out/t_x.log 2>&1; rc=$?
tail -3 gpurun_out/t_x.log
[ $rc -eq 0 ] || exit $rc
for t in 0 1 2 3; do
  echo "GI_X_BLK_LOG2=$t"
  GI_X_BLK_LOG2=$t timeout -k 10 200 python profiles/shard_scaling.py --workload C3 --ns 1,8 --reps 5 > gpurun_out/bl_$t.log 2>&1 || { tail -5 gpurun_out/bl_$t.log; exit 1; }
  grep '"n"' gpurun_out/bl_$t.log | cut -c1-120
done
bash profiles/ab_env.sh C4,C5 GI_X_BLK_LOG2=0 GI_X_BLK_LOG2=2
