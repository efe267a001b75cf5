#!/bin/bash
# A/B of kernel variants x environment settings:  profiles/abx.sh <workloads,comma> <spec>...
#   spec = <variant>[:ENV=v[,ENV=v...]]   variant "default" = libgi.so, else _variants/libgi_<v>.so
# Each variant's Mode X frames are first checked bit for bit against the oracle (GPU parity subset,
# GI_LIB=<variant>); then one bench line per workload (kernel ms from the bench's HIP events).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
WL=$1; shift
declare -A CHECKED
for SPEC in "$@"; do
  V=${SPEC%%:*}; E=""; [[ "$SPEC" == *:* ]] && E=${SPEC#*:}; E=${E//,/ }
  if [ "$V" = default ]; then LIB=$R/2019global_amd/libgi.so; else LIB=$R/2019global_amd/_variants/libgi_$V.so; fi
  if [ -z "${CHECKED[$V]}" ]; then
    GI_LIB=$LIB timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_mode_x_mirror.py -m gpu -x -q \
      --timeout 200 --timeout-method thread -k "mode_x or sharded or mirror" > gpurun_out/abx_t_$V.log 2>&1 \
      || { echo "PARITY FAIL $V"; tail -5 gpurun_out/abx_t_$V.log; exit 1; }
    echo "parity ok $V: $(tail -1 gpurun_out/abx_t_$V.log)"; CHECKED[$V]=1
  fi
  for W in ${WL//,/ }; do
    env GI_LIB=$LIB $E timeout -k 10 300 python bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/abx_$W.log 2>&1 || { tail -5 gpurun_out/abx_$W.log; exit 1; }
    python - "$W" "$SPEC" <<'PY'
import json,sys; d=json.loads(open(f"gpurun_out/abx_{sys.argv[1]}.log").read().strip().splitlines()[-1])
r=d["roofline"]; s=d.get("schedule",{}); b=s.get("blocks",{})
bl=" ".join("%s=%d/%.2f"%(k[:4],v["iterations"]//1000,v["lane_fill"]) for k,v in b.items())
print("%-26s %-5s kern_ms %8.3f ms %8.3f it %s trav_fill %s %s longest %s" % (sys.argv[2], sys.argv[1], r["kernel_ms"], d["ms_per_step"], s.get("wave_iterations"), s.get("trav_lane_fill"), bl, s.get("longest_path",{}).get("ms")), flush=True)
PY
  done
done
