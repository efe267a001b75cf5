#!/bin/bash
# Round-2 start: GPU suite + default bench line on a fresh box (same HEAD as round 1's end).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/r02_base
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_base/gpu_tests.log 2>&1 || { tail -20 gpurun_out/r02_base/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r02_base/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r02_base/bench.json 2> gpurun_out/r02_base/bench.err || { tail -5 gpurun_out/r02_base/bench.err; exit 1; }
tail -1 gpurun_out/r02_base/bench.json
for W in C4 R-C4 R-C3; do
  timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline --steps 5 > gpurun_out/r02_base/bench_$W.json 2>/dev/null || exit 1
  tail -1 gpurun_out/r02_base/bench_$W.json | cut -c1-400
done
