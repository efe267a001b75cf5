cd $GRAFT_REPO_ROOT
bash profiles/r06.sh suite; S=$?
echo "suite rc $S"
if [ $S -ne 0 ] && [ $S -ne 1 ]; then exit $S; fi
GI_LIB=$GRAFT_REPO_ROOT/2019global_amd/_variants/libgi_r05head.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 250 --timeout-method thread -k sparse_tile_column > gpurun_out/r06_oldlib_strip.log 2>&1; R=$?
echo "old-lib strip rc $R"; grep -E "PASSED|FAILED|^E " gpurun_out/r06_oldlib_strip.log | head -8
if [ $R -ne 0 ] && [ $R -ne 1 ]; then exit $R; fi
STEPS=10 bash profiles/r06.sh ab C3,C2 default r05head en4 w5en || exit $?
STEPS=10 bash profiles/r06.sh ab C4,C5,R-C4 default r05head
