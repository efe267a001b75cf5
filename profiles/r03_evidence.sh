#!/bin/bash
# round 3 evidence at HEAD: rocprofv3 kernel stats + PMC (C3, C4, C5, R-C4), per-rank share
# probes (C3, C4, C5), and the default bench line with its CPU baselines
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash profiles/profile.sh r03 C3 C4 C5 R-C4 || exit 1
for W in C3 C4 C5; do
  timeout -k 10 300 python profiles/shard_scaling.py --workload $W --ns 1,2,4,8 --reps 3 > gpurun_out/r03_shard_scaling_${W,,}.jsonl 2>gpurun_out/shard_$W.err || { tail -3 gpurun_out/shard_$W.err; exit 1; }
  tail -1 gpurun_out/r03_shard_scaling_${W,,}.jsonl
done
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_bench_c3.log 2>&1 || { tail -5 gpurun_out/r03_bench_c3.log; exit 1; }
grep '"metric"' gpurun_out/r03_bench_c3.log | tail -1 > gpurun_out/r03_bench_c3.json
python3 -c "import json; d=json.load(open('gpurun_out/r03_bench_c3.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
