# Mode X own-plane leaf skip: the whole GPU suite, then A/B against the previous commit's library
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_t16.log 2>&1; S=$?
tail -2 gpurun_out/r06_t16.log; echo "suite rc $S"
if [ $S -ne 0 ]; then grep -E "^FAILED|^E " gpurun_out/r06_t16.log | head -20; exit $S; fi
STEPS=10 bash profiles/r06.sh ab C3,C2,X-zoo,X-main,C4 default prev || exit $?
