cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "mode_x_bit_exact or forms_bit_identical or spp_runs or mirror or whole_frame" > gpurun_out/r06_t4.log 2>&1; S=$?
tail -2 gpurun_out/r06_t4.log; echo "tests rc $S"
if [ $S -ne 0 ]; then grep -E "^FAILED|^E " gpurun_out/r06_t4.log | head; exit $S; fi
GI_LIB=$GRAFT_REPO_ROOT/2019global_amd/_variants/libgi_stepprobe.so timeout -k 10 300 python3 profiles/path_latency.py --workload C4 > gpurun_out/r06_c4_stepprobe.jsonl 2> gpurun_out/r06_c4_stepprobe.err; echo "probe rc $?"
cut -c1-600 gpurun_out/r06_c4_stepprobe.jsonl
STEPS=10 bash profiles/r06.sh ab C3,C2,X-zoo,C5 default head
