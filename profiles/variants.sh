#!/bin/bash
# Benchmarks kernel build variants (2019global_amd/_variants/libgi_<name>.so, built by
# `python 2019global_amd/build.py --variant <name> DEFINE...`) against the default libgi.so.
#   profiles/variants.sh <workloads, comma separated> <variant names...>   ("default" = libgi.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
WL=$1; shift
for V in "$@"; do
  if [ "$V" = default ]; then LIB=$R/2019global_amd/libgi.so; else LIB=$R/2019global_amd/_variants/libgi_$V.so; fi
  for W in ${WL//,/ }; do
    GI_LIB=$LIB timeout -k 10 300 python bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/var_$W.log 2>&1 || { tail -5 gpurun_out/var_$W.log; exit 1; }
    python - "$W" "$V" <<'PY'
import json,sys; d=json.loads(open(f"gpurun_out/var_{sys.argv[1]}.log").read().strip().splitlines()[-1])
r=d["roofline"]; n=d["config"]["rays_per_frame"]; print("%-8s %-4s Mray/s %9.1f kern_ms %8.3f nodes/ray %.2f prims/ray %.2f" % (sys.argv[2], sys.argv[1], d["value"], r["kernel_ms"], r["node_visits"]/n, r["prim_tests"]/n))
PY
  done
done
