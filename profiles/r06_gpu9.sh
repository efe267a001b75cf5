cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/2019global_amd/_variants
GI_LIB=$V/libgi_coopall.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "mode_r or soup100k or sparse_tile or large_scene or kernels_frame or whole_frame_vs_reference or golden or multi or shard" > gpurun_out/r06_t9.log 2>&1; S=$?
tail -2 gpurun_out/r06_t9.log; echo "coopall tests rc $S"
if [ $S -ne 0 ]; then grep -E "^FAILED|^E " gpurun_out/r06_t9.log | head; exit $S; fi
STEPS=10 bash profiles/r06.sh ab R-C4,R-C3 default coopall || exit $?
for V2 in default coop8; do
  if [ $V2 = default ]; then L=$GRAFT_REPO_ROOT/2019global_amd/libgi.so; else L=$V/libgi_$V2.so; fi
  GI_LIB=$L timeout -k 10 300 python3 profiles/shard_scaling.py --workload R-C4 > gpurun_out/r06_shard_rc4_$V2.jsonl 2>&1 || exit 1
  echo $V2; tail -1 gpurun_out/r06_shard_rc4_$V2.jsonl | cut -c1-400
done
