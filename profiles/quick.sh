#!/bin/bash
# quick GPU iteration: Mode X parity subset + C2/C3/C4 bench lines (no cpu baseline)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "mode_x or sharded or bands" > gpurun_out/t_x.log 2>&1; rc=$?
tail -2 gpurun_out/t_x.log
[ $rc -eq 0 ] || exit $rc
for W in C2 C3 C4 "$@"; do
  timeout -k 10 300 python bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$W.log 2>&1 || { tail -5 gpurun_out/bench_$W.log; exit 1; }
  python - "$W" <<'PY'
import json,sys; d=json.loads(open(f"gpurun_out/bench_{sys.argv[1]}.log").read().strip().splitlines()[-1])
r=d["roofline"]; print(sys.argv[1], "Mray/s", d["value"], "ms", d["ms_per_step"], "kern_ms", r["kernel_ms"], "nodes/ray %.2f prims/ray %.2f" % (r["node_visits"]/d["config"]["rays_per_frame"], r["prim_tests"]/d["config"]["rays_per_frame"]), "alg GB/s", r["achieved"])
PY
done
