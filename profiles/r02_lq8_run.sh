#!/bin/bash
# Leaf-phase threshold sweep (GI_X_LEAF8) for the LQ variant on C5 and the 1k soup
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash profiles/ab.sh C5,X-soup1000 default || exit 1
for l in 1 2 3 4 5; do GI_X_LEAF8=$l bash profiles/ab.sh C5,X-soup1000 lq | sed "s/^/LEAF8=$l /" || exit 1; done
