#!/bin/bash
# round 3, last change (no load after a leaf's last record in long launches): GPU suite, C5
# rocprofv3 stats + PMC, C5 share probe, C5 and C4 bench lines
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash profiles/gpu_tests.sh r03final2 || exit 1
bash profiles/profile.sh r03 C5 || exit 1
cp gpurun_out/r03prof/r03_c5_pmc.json profiles/
timeout -k 10 300 python profiles/shard_scaling.py --workload C5 --ns 1,2,4,8 --reps 3 > gpurun_out/r03_shard_scaling_c5.jsonl 2>gpurun_out/shard_C5.err || { tail -3 gpurun_out/shard_C5.err; exit 1; }
tail -1 gpurun_out/r03_shard_scaling_c5.jsonl
bash profiles/benchall.sh C5 C4
