#!/bin/bash
# Round-2 evidence at HEAD: GPU suite, the default bench line (C3, with CPU baselines), every
# workload's line, rocprofv3 kernel stats + PMC for C3/C4/C5/R-C4, and the C5 per-rank share probe.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/r02final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02final/gpu_tests.log 2>&1 || { tail -20 gpurun_out/r02final/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r02final/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r02final/bench_c3.json 2> gpurun_out/r02final/bench_c3.err || { tail -5 gpurun_out/r02final/bench_c3.err; exit 1; }
tail -1 gpurun_out/r02final/bench_c3.json | cut -c1-300
bash profiles/benchall.sh C2 C3 C4 C5 R-C3 R-C4 R-main X-main X-zoo X-soup1000 > gpurun_out/r02final/benchall.txt 2>&1 || { cat gpurun_out/r02final/benchall.txt; exit 1; }
cat gpurun_out/r02final/benchall.txt
for f in gpurun_out/all_*.json; do cp $f gpurun_out/r02final/; done
bash profiles/r02_profile.sh C3 C4 C5 R-C4 || exit 1
timeout -k 10 400 python -u profiles/shard_scaling.py --workload C5 --reps 3 > gpurun_out/r02final/shard_C5.jsonl 2>/dev/null || exit 1
tail -1 gpurun_out/r02final/shard_C5.jsonl
