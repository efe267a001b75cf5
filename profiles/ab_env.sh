#!/bin/bash
# A/B of environment settings on bench workloads: profiles/ab_env.sh <workloads> "<ENV=..>" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
WL=$1; shift
for W in ${WL//,/ }; do
  for E in "$@"; do
    env $E timeout -k 10 300 python bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/abe_$W.log 2>&1 || { tail -5 gpurun_out/abe_$W.log; exit 1; }
    python - "$W" "$E" <<'PY'
import json,sys; d=json.loads(open(f"gpurun_out/abe_{sys.argv[1]}.log").read().strip().splitlines()[-1])
r=d["roofline"]; s=d.get("schedule",{}); print("%-22s %-6s Mray/s %9.1f ms %8.3f kern_ms %8.3f trav_fill %s h_fill %s longest %s" % (sys.argv[2], sys.argv[1], d["value"], d["ms_per_step"], r["kernel_ms"], s.get("trav_lane_fill"), s.get("handler_lane_fill"), s.get("longest_path")), flush=True)
PY
  done
done
