#!/bin/bash
# Profile evidence for a round: rocprofv3 kernel-trace --stats + separate PMC passes (incl. FP64
# VALU counters) of the bench command, per workload, summarised to
# gpurun_out/<tag>prof/<tag>_<w>_pmc.json + <tag>_<w>_kernel_stats.csv (copy into profiles/).
#   profiles/profile.sh <tag, e.g. r03> C3 C4 R-C4 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
TAG=$1; shift
mkdir -p gpurun_out/${TAG}prof
for W in "$@"; do
  w=$(echo $W | tr A-Z a-z)
  # the dominant kernel (k_mode_x, k_wf_bounce or k_mode_r) is found by summarize.py; the wavefront
  # form's figures are per frame (3 timed + 1 warm-up frames)
  bash profiles/run_profile.sh ${w}_${TAG} --workload $W --steps 3 --warmup 1 || { echo "profile $W failed"; exit 1; }
  python3 profiles/summarize.py gpurun_out/prof_${w}_${TAG} $W auto gpurun_out/${TAG}prof/${TAG}_${w}_pmc.json 4 || exit 1
  cp gpurun_out/prof_${w}_${TAG}/trace/run_kernel_stats.csv gpurun_out/${TAG}prof/${TAG}_${w}_kernel_stats.csv
done
echo profiles done
