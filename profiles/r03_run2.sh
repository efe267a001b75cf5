#!/bin/bash
# round 3: Mode R memo A/B, then the GPU suite and one bench line per workload (host paths included)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for V in default m32 m128 ns16 default; do
  if [ "$V" = default ]; then LIB=$R/2019global_amd/libgi.so; else LIB=$R/2019global_amd/_variants/libgi_$V.so; fi
  GI_LIB=$LIB timeout -k 10 200 python bench.py --workload R-C4 --steps 5 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/rm_$V.log 2>&1 || { tail -3 gpurun_out/rm_$V.log; exit 1; }
  echo "$V $(tail -1 gpurun_out/rm_$V.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_ms"], d["roofline"]["node_visits"])')"
done
bash profiles/gpu_tests.sh r03b || exit 1
for W in C3 C2 C4 C5 R-C3 R-C4 R-main X-main X-zoo X-soup1000; do
  timeout -k 10 300 python bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/all_$W.log 2>&1 || { tail -n 5 gpurun_out/all_$W.log; exit 1; }
  grep '"metric"' gpurun_out/all_$W.log | tail -n 1 > gpurun_out/all_$W.json
  python3 - "$W" <<'PY'
import json,sys; d=json.load(open(f"gpurun_out/all_{sys.argv[1]}.json"))
r=d["roofline"]; n=d["config"]["rays_per_frame"]
print("%-10s Mray/s(traced) %9.1f ms %8.3f kern_ms %8.3f frac %.3f nodes/ray %.2f prims/ray %.2f" % (sys.argv[1], d["value"], d["ms_per_step"], r["kernel_ms"], r["frac"], r["node_visits"]/n, r["prim_tests"]/n))
print("   host:", json.dumps(d.get("host_path",{}).get("ms_per_frame")), d.get("host_path",{}).get("error",""))
PY
done
