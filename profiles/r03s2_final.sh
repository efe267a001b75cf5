#!/bin/bash
# round 3, last session: GPU suite, then C4/C5 rocprofv3 stats + PMC, share probes and bench lines
# at HEAD (handler threshold 4/8 for the 100k soup)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash profiles/gpu_tests.sh r03final || exit 1
bash profiles/profile.sh r03 C4 C5 || exit 1
for W in C4 C5; do
  timeout -k 10 300 python profiles/shard_scaling.py --workload $W --ns 1,2,4,8 --reps 3 > gpurun_out/r03_shard_scaling_${W,,}.jsonl 2>gpurun_out/shard_$W.err || { tail -3 gpurun_out/shard_$W.err; exit 1; }
  tail -1 gpurun_out/r03_shard_scaling_${W,,}.jsonl
done
bash profiles/benchall.sh C4 C5 C3
