#!/bin/bash
# round 4: where the wavefront form's time goes -- per-dispatch kernel trace of C3 (both forms) and
# three PMC passes each (instructions, cycles, lane utilisation)
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r04wfp; mkdir -p $O; export TMPDIR=/tmp
W=${1:-C3}
cd /tmp
for F in ${FORMS:-wf mega}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$F -o run -- python3 $R/profiles/wf_probe.py --steps 2 --warmup 1 --forms $F $W > $O/trace_$F.log 2>&1 || { echo "trace $F failed"; tail -5 $O/trace_$F.log; exit 1; }
  i=0
  for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY" \
           "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $O/pmc_${F}_$i -o run -- python3 $R/profiles/wf_probe.py --steps 2 --warmup 1 --forms $F $W > $O/pmc_${F}_$i.log 2>&1 || { echo "pmc $F $i failed"; tail -5 $O/pmc_${F}_$i.log; exit 1; }
  done
done
echo done
