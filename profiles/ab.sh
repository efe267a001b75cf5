#!/bin/bash
# A/B of kernel build variants on bench workloads (kernel time from the bench's HIP events).
#   profiles/ab.sh <workloads, comma separated> <variant names...>   ("default" = libgi.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
WL=$1; shift
for W in ${WL//,/ }; do
  for V in "$@"; do
    if [ "$V" = default ]; then LIB=$R/2019global_amd/libgi.so; else LIB=$R/2019global_amd/_variants/libgi_$V.so; fi
    GI_LIB=$LIB timeout -k 10 300 python bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/ab_$W.log 2>&1 || { tail -5 gpurun_out/ab_$W.log; exit 1; }
    python - "$W" "$V" <<'PY'
import json,sys; d=json.loads(open(f"gpurun_out/ab_{sys.argv[1]}.log").read().strip().splitlines()[-1])
r=d["roofline"]; s=d.get("schedule",{}); print("%-8s %-8s Mray/s %9.1f ms %8.3f kern_ms %8.3f trav_fill %s h_fill %s longest %s" % (sys.argv[2], sys.argv[1], d["value"], d["ms_per_step"], r["kernel_ms"], s.get("trav_lane_fill"), s.get("handler_lane_fill"), s.get("longest_path")), flush=True)
PY
  done
done
