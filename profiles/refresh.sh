#!/bin/bash
# Round evidence on one GPU box: parity suite, default bench line (with CPU baselines), and the
# rocprofv3 kernel-trace + PMC summaries for C3 and C4 (profiles/run_profile.sh + summarize.py).
#   profiles/refresh.sh <tag>     -> gpurun_out/refresh_<tag>/...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
TAG=${1:-r01}
OUT=gpurun_out/refresh_$TAG; mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -q > $OUT/gpu_tests.log 2>&1 || { tail -20 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -5 $OUT/bench_default.err; exit 1; }
tail -1 $OUT/bench_default.json
for W in C3 C4; do
  w=$(echo $W | tr A-Z a-z)
  bash profiles/run_profile.sh ${w}_$TAG --workload $W --steps 3 --warmup 1 || exit 1
  python3 profiles/summarize.py gpurun_out/prof_${w}_$TAG $W k_mode_x $OUT/${TAG}_${w}_pmc.json || exit 1
  cp gpurun_out/prof_${w}_$TAG/trace/run_kernel_stats.csv $OUT/${TAG}_${w}_kernel_stats.csv
done
for W in C4 C5; do
  w=$(echo $W | tr A-Z a-z)
  timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail -5 $OUT/bench_$w.err; exit 1; }
done
timeout -k 10 300 python profiles/shard_scaling.py > $OUT/shard_scaling_c3.log 2>&1 || { tail -5 $OUT/shard_scaling_c3.log; exit 1; }
grep '^{"n"' $OUT/shard_scaling_c3.log > $OUT/${TAG}_shard_scaling_c3.jsonl
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 > $OUT/${TAG}_rehearsal_n2_gloo.log 2>&1 || { tail -5 $OUT/${TAG}_rehearsal_n2_gloo.log; exit 1; }
tail -1 $OUT/${TAG}_rehearsal_n2_gloo.log
echo refresh done
