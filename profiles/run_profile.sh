#!/bin/bash
# Collects the rocprofv3 evidence under gpurun_out/prof_<tag>/ on the GPU box:
#   kernel-trace --stats of the bench command, then separate --pmc passes (never combined with
#   any trace domain, per the pool's rules).  Usage: profiles/run_profile.sh <tag> <bench args...>
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --no-cpu-baseline --no-host-path "$@" > $OUT/trace.log 2>&1 || exit $?
i=0
# PMC_PASSES="pass;pass;...": other counter passes (e.g. the memory-pipeline set of profiles/r05.sh mem)
if [ -n "$PMC_PASSES" ]; then IFS=';' read -ra PASSES <<< "$PMC_PASSES"; else PASSES=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY" \
         "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
         "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP32 GRBM_GUI_ACTIVE"); fi
for P in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc$i -o run -- python3 $R/bench.py --no-cpu-baseline --no-host-path "$@" > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed: $P"; exit 1; }
done
echo done
