#!/bin/bash
# Round-2 evidence refresh at HEAD: every workload's bench line, then rocprofv3 kernel stats + PMC
# for C4, C5 and C3 (summaries -> gpurun_out/r02prof/).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/r02prof
bash profiles/benchall.sh C2 C3 C4 C5 R-C3 R-C4 R-main X-main X-zoo X-soup1000 > gpurun_out/r02prof/benchall.txt 2>&1 || { cat gpurun_out/r02prof/benchall.txt; exit 1; }
cat gpurun_out/r02prof/benchall.txt
for f in gpurun_out/all_*.json; do cp $f gpurun_out/r02prof/; done
bash profiles/r02_profile.sh C4 C5 C3
