set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "mode_x or sharded or anchored" > gpurun_out/t_x.log 2>&1; rc=$?
tail -3 gpurun_out/t_x.log
[ $rc -eq 0 ] || exit $rc
bash profiles/ab.sh C4,C5,C3,X-soup1000 default nst0
