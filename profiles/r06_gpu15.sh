# k_rf_reach with the launch-chosen lanes per hit: parity, R-C4/R-C3 bench, eighth-share against G=1, probe
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "lane_groups or mode_r or soup100k or sparse_tile or large_scene or golden or shard" > gpurun_out/r06_t15.log 2>&1; S=$?
tail -2 gpurun_out/r06_t15.log; echo "tests rc $S"
if [ $S -ne 0 ]; then grep -E "^FAILED|^E " gpurun_out/r06_t15.log | head; exit $S; fi
for W in R-C4 R-C3; do
  timeout -k 10 200 python3 bench.py --workload $W --steps 10 --warmup 2 --no-cpu-baseline --no-host-path > gpurun_out/r06_b15_$W.json 2> gpurun_out/r06_b15_$W.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r06_b15_$W.json').read().strip().splitlines()[-1]); print('$W kernel %.4f ms frame %.4f ms' % (d['roofline']['kernel_ms'], d['ms_per_step']))"
done
for G in 0 1; do
  GI_RF_GROUP=$G timeout -k 10 300 python3 profiles/shard_scaling.py --workload R-C4 > gpurun_out/r06_shard_rc4_g$G.jsonl 2>&1 || exit 1
  echo "group $G"; tail -1 gpurun_out/r06_shard_rc4_g$G.jsonl | cut -c1-500
done
GI_LIB=$GRAFT_REPO_ROOT/2019global_amd/_variants/libgi_reachprobe.so timeout -k 10 300 python3 -u profiles/reach_probe.py soup100000 > gpurun_out/reach_probe_auto.jsonl 2> gpurun_out/reach_probe_auto.err || exit 1
echo probe done
