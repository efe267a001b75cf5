#!/bin/bash
# round 4 evidence at HEAD, part A: GPU suite, rocprofv3 kernel stats + PMC of the default forms
# (C3/C2 k_seg, C4/C5 k_mode_x, R-C4 k_mode_r_split), shard-scaling probes, bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04ev; mkdir -p $O
[ -n "$SKIP_SUITE" ] || timeout -k 10 400 python3 -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -20 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 1000 bash profiles/profile.sh r04 ${WLS:-C3 C2 C4 R-C4 C5} > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
for W in C3 C5 C4; do
  timeout -k 10 300 python3 profiles/shard_scaling.py --workload $W > $O/shard_$W.jsonl 2>&1 || { tail -5 $O/shard_$W.jsonl; exit 1; }
  tail -1 $O/shard_$W.jsonl
done
echo evidence A done
