#!/bin/bash
# Mode X leaf-size sweep (GI_XLEAF_MAX) on C2/C3/C4, 3 timed frames each
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for LM in "$@"; do for W in C2 C3 C4; do
  GI_XLEAF_MAX=$LM timeout -k 10 300 python bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ls_$W.log 2>&1 || { tail -5 gpurun_out/ls_$W.log; exit 1; }
  python - "$W" "$LM" <<'PY'
import json,sys; d=json.loads(open(f"gpurun_out/ls_{sys.argv[1]}.log").read().strip().splitlines()[-1])
r=d["roofline"]; n=d["config"]["rays_per_frame"]; print("leaf", sys.argv[2], sys.argv[1], "Mray/s", d["value"], "kern_ms", r["kernel_ms"], "nodes/ray %.2f prims/ray %.2f" % (r["node_visits"]/n, r["prim_tests"]/n))
PY
done; done
