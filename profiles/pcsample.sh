#!/bin/bash
# PC sampling (rocprofv3 host-trap, time-based) of one bench workload's frames: where the waves of
# the dominant kernel spend their time, instruction by instruction.
#   profiles/pcsample.sh <workload> <tag> [interval_us]  -> gpurun_out/pcs_<tag>/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
W=$1; TAG=$2; IV=${3:-1}
OUT=$R/gpurun_out/pcs_$TAG
mkdir -p $OUT
cd /tmp
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval $IV --output-format csv -d $OUT/raw -o run -- \
  python3 $R/bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > $OUT/run.log 2>&1
rc=$?
ls -R $OUT/raw | head -20
exit $rc
