#!/bin/bash
# LQ on by default (quantised-node scenes, long launches): Mode X parity, every Mode X workload
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "mode_x or soup or handoff or shard" > gpurun_out/t_lq.log 2>&1; rc=$?
tail -3 gpurun_out/t_lq.log
[ $rc -eq 0 ] || exit $rc
bash profiles/ab.sh C5,C4,X-soup1000,C3 default || exit 1
