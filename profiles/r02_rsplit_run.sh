set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "mode_r or golden or trace or kat or soup100k or band or cancel or dropin or multi or sharded" > gpurun_out/t_r.log 2>&1; rc=$?
tail -3 gpurun_out/t_r.log
[ $rc -eq 0 ] || exit $rc
bash profiles/ab_env.sh R-C4,R-C3,R-main GI_R_SPLIT=-1 GI_R_SPLIT=0 GI_R_SPLIT=1
