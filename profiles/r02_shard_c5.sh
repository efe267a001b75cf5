#!/bin/bash
# Per-rank share timing on the 8-GPU config's own workload (C5) and on C4.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/r02_shard
for W in C5 C4; do
  timeout -k 10 400 python -u profiles/shard_scaling.py --workload $W --reps 3 > gpurun_out/r02_shard/shard_$W.jsonl 2> gpurun_out/r02_shard/shard_$W.err || { tail -5 gpurun_out/r02_shard/shard_$W.err; exit 1; }
  cat gpurun_out/r02_shard/shard_$W.jsonl
done
