# k_rf_reach head / tail split (GI_RF_SPLIT, experiment): parity at one split, then R-C4 per split
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06split
GI_RF_SPLIT=2048 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "lane_groups or soup100k or mode_r_vs_reference" > gpurun_out/r06split/parity.log 2>&1 || { tail -20 gpurun_out/r06split/parity.log; exit 1; }
tail -1 gpurun_out/r06split/parity.log
for REP in 1 2; do
for S in 0 1024 1536 2048 2560 3072; do
  GI_RF_SPLIT=$S timeout -k 10 200 python3 bench.py --workload R-C4 --steps 10 --warmup 2 --no-cpu-baseline --no-host-path > gpurun_out/r06split/rc4_$S.json 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r06split/rc4_$S.json').read().strip().splitlines()[-1]); print('split $S kernel %.4f ms frame %.4f ms' % (d['roofline']['kernel_ms'], d['ms_per_step']))"
done
done
