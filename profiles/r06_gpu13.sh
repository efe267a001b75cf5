cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/2019global_amd/_variants
GI_LIB=$V/libgi_defer16.so timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "mode_x_bit_exact or forms_bit_identical or whole_frame or spp_runs or mirror or ragged" > gpurun_out/r06_t13.log 2>&1; S=$?; echo "defer16 tests rc $S"; tail -1 gpurun_out/r06_t13.log
if [ $S -ne 0 ]; then grep -E "^FAILED|^E " gpurun_out/r06_t13.log | head; exit $S; fi
STEPS=10 bash profiles/r06.sh ab C3,C2,X-zoo,X-main default defer8 defer16 defer32
