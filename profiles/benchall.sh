#!/bin/bash
# One bench line per workload (no CPU baseline) -> gpurun_out/all_<W>.json; prints a summary row each.
#   profiles/benchall.sh C2 C3 C4 R-C3 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for W in "$@"; do
  timeout -k 10 300 python bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/all_$W.log 2>&1 || { tail -n 5 gpurun_out/all_$W.log; exit 1; }
  grep '"metric"' gpurun_out/all_$W.log | tail -n 1 > gpurun_out/all_$W.json
  python3 - "$W" <<'PY'
import json,sys; d=json.load(open(f"gpurun_out/all_{sys.argv[1]}.json"))
r=d["roofline"]; n=d["config"]["rays_per_frame"]
print("%-7s Mray/s %9.1f ms %8.3f kern_ms %8.3f frac %.3f nodes/ray %.2f prims/ray %.2f" % (sys.argv[1], d["value"], d["ms_per_step"], r["kernel_ms"], r["frac"], r["node_visits"]/n, r["prim_tests"]/n))
PY
done
