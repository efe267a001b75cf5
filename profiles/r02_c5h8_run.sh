#!/bin/bash
# C5 with LQ: handler threshold sweep and the per-rank share probe (N = 1, 8)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash profiles/ab_env.sh C5 GI_X_HANDLE8=2 GI_X_HANDLE8=4 || exit 1
timeout -k 10 500 python -u profiles/shard_scaling.py --workload C5 --ns 1,8 --reps 2 > gpurun_out/ss_c5.log 2>&1 || { tail -5 gpurun_out/ss_c5.log; exit 1; }
grep '"n"' gpurun_out/ss_c5.log | cut -c1-150
