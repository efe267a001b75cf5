set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
tail -3 gpurun_out/t_all.log
[ $rc -eq 0 ] || exit $rc
bash profiles/benchall.sh C2 C3 C4 C5 X-zoo X-soup1000 X-main
