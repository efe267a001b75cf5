R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for SPEC in "default:" "spec:GI_X_HANDLE8=6" "spec:GI_X_HANDLE8=8"; do
  V=${SPEC%%:*}; E=${SPEC#*:}
  if [ "$V" = default ]; then LIB=$R/2019global_amd/libgi.so; else LIB=$R/2019global_amd/_variants/libgi_$V.so; fi
  echo "== $SPEC"
  env GI_LIB=$LIB $E timeout -k 10 200 python profiles/shard_scaling.py --workload C3 --ns 1,8 --reps 3 2>&1 | tail -4 || exit 1
done
timeout -k 10 300 python bench.py --workload C5 --steps 2 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/c5.log 2>&1 || exit 1
tail -1 gpurun_out/c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5', d['roofline']['kernel_ms'], json.dumps(d['schedule']))"
