R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
GI_LIB=$R/2019global_amd/libgi.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "mode_r or reference or soup or dfs or r_" > gpurun_out/rab_t.log 2>&1 || { tail -5 gpurun_out/rab_t.log; exit 1; }
tail -1 gpurun_out/rab_t.log
for V in default rnopf default rnopf; do
  if [ "$V" = default ]; then LIB=$R/2019global_amd/libgi.so; else LIB=$R/2019global_amd/_variants/libgi_$V.so; fi
  for W in R-C4 R-C3; do
  GI_LIB=$LIB timeout -k 10 200 python bench.py --workload $W --steps 5 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/rab.log 2>&1 || { tail -3 gpurun_out/rab.log; exit 1; }
  echo "$V $W $(tail -1 gpurun_out/rab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_ms"], d["roofline"]["node_visits"])')"
  done
done
