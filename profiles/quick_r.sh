#!/bin/bash
# quick Mode R iteration: Mode R parity subset + R-C3 / R-C4 bench lines
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "mode_r or golden or trace or kat or soup100k" > gpurun_out/t_r.log 2>&1; rc=$?
tail -2 gpurun_out/t_r.log
[ $rc -eq 0 ] || exit $rc
for W in R-C3 R-C4 R-main "$@"; do
  timeout -k 10 300 python bench.py --workload $W --steps 5 --warmup 2 --no-cpu-baseline --no-host-path > gpurun_out/bench_$W.log 2>&1 || { tail -5 gpurun_out/bench_$W.log; exit 1; }
  python - "$W" <<'PY'
import json,sys; d=json.loads(open(f"gpurun_out/bench_{sys.argv[1]}.log").read().strip().splitlines()[-1])
r=d["roofline"]; print(sys.argv[1], "Mray/s", d["value"], "ms", d["ms_per_step"], "kern_ms", r["kernel_ms"])
PY
done
