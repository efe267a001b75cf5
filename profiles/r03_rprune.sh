#!/bin/bash
# Mode R rank-ordered line BVH with pruning: Mode R GPU parity subset, then R-C4 / R-C3 bench lines
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "mode_r or split_candidates or raytracer_api or expbox or trace_ray" > gpurun_out/rp_t.log 2>&1 || { echo "PARITY FAIL"; tail -5 gpurun_out/rp_t.log; exit 1; }
echo "parity ok: $(tail -1 gpurun_out/rp_t.log)"
for rep in 1 2; do for W in R-C4 R-C3; do
  timeout -k 10 300 python bench.py --workload $W --steps 5 --warmup 2 --no-cpu-baseline --no-host-path > gpurun_out/rp_$W.log 2>&1 || { tail -5 gpurun_out/rp_$W.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/rp_$W.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$W kern_ms', r['kernel_ms'], 'ms', d['ms_per_step'], 'nodes', r.get('node_visits'), 'prims', r.get('prim_tests'))"
done; done
