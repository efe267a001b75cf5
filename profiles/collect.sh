#!/bin/bash
# Copies a refresh.sh run (gpurun_out/refresh_<tag>/, gpurun_out/prof_*_<tag>/) into profiles/ as the
# round's evidence:  profiles/collect.sh <tag> [round prefix, default r01]
T=$1; P=${2:-r01}; S=gpurun_out/refresh_$T
set -e
cp $S/bench_default.json profiles/${P}_bench_c3.json
for w in c3 c4; do
  cp $S/${T}_${w}_pmc.json profiles/${P}_${w}_pmc.json
  cp $S/${T}_${w}_kernel_stats.csv profiles/${P}_${w}_kernel_stats.csv
done
grep -h '"metric"' gpurun_out/prof_c4_$T/trace.log | tail -n 1 > profiles/${P}_bench_c4.json
tail -n 1 $S/gpu_tests.log > profiles/${P}_gpu_tests.log
[ -f $S/shard_c3.log ] && grep '^{"n"' $S/shard_c3.log > profiles/${P}_shard_scaling_c3.jsonl || true
ls -la profiles/${P}_*
