#!/bin/bash
# Round-2 profile evidence: rocprofv3 kernel-trace --stats + separate PMC passes (incl. FP64 VALU
# counters) for the given workloads, summarised to gpurun_out/r02_<w>_pmc.json + kernel stats.
#   profiles/r02_profile.sh C3 C4 R-C3 R-C4 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/r02prof
for W in "$@"; do
  w=$(echo $W | tr A-Z a-z)
  KERN=k_mode_x; case $W in R-*) KERN=k_mode_r;; esac
  bash profiles/run_profile.sh ${w}_r02 --workload $W --steps 3 --warmup 1 || { echo "profile $W failed"; exit 1; }
  python3 profiles/summarize.py gpurun_out/prof_${w}_r02 $W $KERN gpurun_out/r02prof/r02_${w}_pmc.json || exit 1
  cp gpurun_out/prof_${w}_r02/trace/run_kernel_stats.csv gpurun_out/r02prof/r02_${w}_kernel_stats.csv
done
echo profiles done
