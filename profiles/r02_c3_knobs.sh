#!/bin/bash
# C3 schedule / tree knobs at HEAD: handler threshold and leaf size (bench A/B through ab_env.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash profiles/ab_env.sh C3 GI_X_HANDLE8=8 GI_X_HANDLE8=7 GI_X_HANDLE8=6 GI_X_HANDLE8=5 GI_XLEAF_MAX=2 GI_XLEAF_MAX=3 GI_XLEAF_MAX=6 GI_XLEAF_MAX=8
