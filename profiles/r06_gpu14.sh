# k_rf_reach lane groups (GI_RF_G=4): parity + R-C4/R-C3 A/B, the eighth-share, the per-chunk probe
cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/2019global_amd/_variants
mkdir -p gpurun_out
bash profiles/r06.sh rab default rfg4 || exit $?
for V2 in default rfg4; do
  if [ $V2 = default ]; then L=$GRAFT_REPO_ROOT/2019global_amd/libgi.so; else L=$V/libgi_$V2.so; fi
  GI_LIB=$L timeout -k 10 300 python3 profiles/shard_scaling.py --workload R-C4 > gpurun_out/r06_shard_rc4_$V2.jsonl 2>&1 || exit 1
  echo $V2; tail -1 gpurun_out/r06_shard_rc4_$V2.jsonl | cut -c1-500
done
GI_LIB=$V/libgi_reachprobe_g4.so timeout -k 10 300 python3 -u profiles/reach_probe.py soup100000 > gpurun_out/reach_probe_g4.jsonl 2> gpurun_out/reach_probe_g4.err || exit 1
echo probe done
