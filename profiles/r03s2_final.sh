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
cp gpurun_out/r03prof/r03_c4_pmc.json gpurun_out/r03prof/r03_c5_pmc.json profiles/   # the bench lines cite them
bash profiles/benchall.sh C4 C5 || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_bench_c3.log 2>&1 || { tail -5 gpurun_out/r03_bench_c3.log; exit 1; }
grep '"metric"' gpurun_out/r03_bench_c3.log | tail -1 > gpurun_out/r03_bench_c3.json
python3 -c "import json; d=json.load(open('gpurun_out/r03_bench_c3.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
