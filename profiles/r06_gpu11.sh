cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/2019global_amd/_variants
bash profiles/r06_ktrace_shard.sh R-C4 8 default coop8 || exit $?
STEPS=10 bash profiles/r06.sh ab C3,C2,C4,C5,R-C4 default ilp maxmemoryclause || exit $?
GI_LIB=$V/libgi_ilp.so timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "mode_x_bit_exact or forms_bit_identical or whole_frame or spp_runs" > gpurun_out/r06_t11.log 2>&1; echo "ilp tests rc $?"; tail -1 gpurun_out/r06_t11.log
