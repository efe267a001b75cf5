cd $GRAFT_REPO_ROOT
bash profiles/r06.sh suite; S=$?
echo "suite rc $S"
if [ $S -ne 0 ] && [ $S -ne 1 ]; then exit $S; fi
GI_LIB=$GRAFT_REPO_ROOT/2019global_amd/_variants/libgi_r05head.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 250 --timeout-method thread -k sparse_tile_column > gpurun_out/r06_oldlib_strip.log 2>&1; R=$?
echo "old-lib strip rc $R"; tail -3 gpurun_out/r06_oldlib_strip.log
if [ $R -ne 0 ] && [ $R -ne 1 ]; then exit $R; fi
timeout -k 10 400 python3 bench.py --steps 20 --warmup 2 > gpurun_out/r06_bench_c3.json 2> gpurun_out/r06_bench_c3.err; B=$?
echo "bench rc $B"; tail -c 600 gpurun_out/r06_bench_c3.json
exit $S
