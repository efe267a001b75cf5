set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
tail -3 gpurun_out/t_all.log
[ $rc -eq 0 ] || exit $rc
bash profiles/ab_env.sh C5,C4,X-soup1000 GI_X_CNODE=1 GI_X_CNODE=0
