#!/bin/bash
# Benchmarks run-time tuning knobs (environment variables read by libgi) on chosen workloads.
#   profiles/knobs.sh <workloads, comma separated> "<VAR=V[,VAR=V...]>" ...   ("-" = defaults)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
WL=$1; shift
for K in "$@"; do
  ENVS=(); [ "$K" != "-" ] && IFS=',' read -ra ENVS <<< "$K"
  for W in ${WL//,/ }; do
    env "${ENVS[@]}" timeout -k 10 300 python bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/knob_$W.log 2>&1 || { tail -5 gpurun_out/knob_$W.log; exit 1; }
    python - "$W" "$K" <<'PY'
import json,sys; d=json.loads(open(f"gpurun_out/knob_{sys.argv[1]}.log").read().strip().splitlines()[-1])
r=d["roofline"]; n=d["config"]["rays_per_frame"]; print("%-28s %-4s Mray/s %9.1f kern_ms %8.3f nodes/ray %.2f prims/ray %.2f" % (sys.argv[2], sys.argv[1], d["value"], r["kernel_ms"], r["node_visits"]/n, r["prim_tests"]/n))
if "schedule" in d: print("    ", json.dumps(d["schedule"]))
PY
  done
done
