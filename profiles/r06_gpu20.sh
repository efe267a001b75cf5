# ExpBox face test without the normalisation when the parallel test is clear: Mode R parity subset,
# then R-C4 / R-C3 / R-main A/B against the previous commit's library
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "mode_r or golden or soup100k or sparse_tile or large_scene or kernels_frame or whole_frame_vs_reference or lane_groups or box or expbox or kat" > gpurun_out/r06_t20.log 2>&1; S=$?
tail -2 gpurun_out/r06_t20.log; echo "tests rc $S"
if [ $S -ne 0 ]; then grep -E "^FAILED|^E " gpurun_out/r06_t20.log | head; exit $S; fi
STEPS=10 bash profiles/r06.sh ab R-C4,R-C3,R-main default prev || exit $?
