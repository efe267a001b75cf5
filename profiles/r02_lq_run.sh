#!/bin/bash
# Leaf postponement (GI_X_LEAFQ variant build): Mode X parity with the variant, then A/B on the
# HBM-resident workloads and the leaf-phase threshold (GI_X_LEAF8)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
LQ=$GRAFT_REPO_ROOT/2019global_amd/_variants/libgi_lq.so
GI_LIB=$LQ timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "mode_x or soup or handoff or shard" > gpurun_out/t_lq.log 2>&1; rc=$?
tail -3 gpurun_out/t_lq.log
[ $rc -eq 0 ] || exit $rc
bash profiles/ab.sh C4,X-soup1000,C5 default lq || exit 1
for l in 4 6; do GI_X_LEAF8=$l bash profiles/ab.sh C4,C5 lq | sed "s/^/LEAF8=$l /" || exit 1; done
