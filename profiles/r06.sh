#!/bin/bash
# Round-6 GPU runs, one entry point (run from gpurun: paths relative to $GRAFT_REPO_ROOT).
#   profiles/r06.sh suites [forms]             GPU suite with the default form choice, then with each
#                                              Mode X form forced (GI_X_WF=0 persistent, 1 wavefront,
#                                              2 segment-synchronous; default "2 1 0")
#   profiles/r06.sh formab <wls,> <spec> ...   the Mode X forms per workload and kernel variant, every
#                                              form's frame checked bit for bit against the first
#                                              (FORMS=mega,wf,seg selects the forms)
#   profiles/r06.sh rab <spec> ...             Mode R: parity subset, then R-C4 / R-C3 bench lines
#   profiles/r06.sh benchq <wls,> [steps]      quick bench lines (kernel ms, schedule block)
#   profiles/r06.sh tk <pytest -k expr> [wls,]  GPU tests selected by -k, then quick bench lines
#   profiles/r06.sh ktrace <wls,> <spec> ...    rocprofv3 --kernel-trace --stats of the bench (5 frames):
#                                              every kernel's calls and average us
#   profiles/r06.sh ab <wls,> <spec> ...        bench lines (kernel ms, ms/frame) per workload and spec,
#                                              interleaved twice (spec order ABAB) against drift
#   profiles/r06.sh mem <wls,> <spec> ...       memory-pipeline PMC passes (L2 latency at the L1, TA/TCP
#                                              stalls, instruction cache) of the dominant kernel
#   profiles/r06.sh evidence 1|2|forms         1: GPU suite + rocprofv3 stats/PMC of the default kernels
#                                              (C3 C2 C4 R-C4 C5, or $WLS); 2: shard probes, bench lines
#                                              of every workload, the C3 bench with its CPU baseline, the
#                                              N = 8 gloo rehearsal; forms: the forced-form profiles (C3
#                                              under k_mode_x and the wavefront form, C5 under the
#                                              wavefront and segment forms)
# A <spec> is <variant>[:ENV=v,...]: variant "default" = 2019global_amd/libgi.so, else
# 2019global_amd/_variants/libgi_<variant>.so (python -m 2019global_amd.build --variant NAME DEFINES).
set -o pipefail
cd $GRAFT_REPO_ROOT
lib() { if [ "$1" = default ]; then echo $GRAFT_REPO_ROOT/2019global_amd/libgi.so; else echo $GRAFT_REPO_ROOT/2019global_amd/_variants/libgi_$1.so; fi; }
what=$1; shift
case $what in
suite)
  O=gpurun_out/r06suite; mkdir -p $O
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/suite.log 2>&1; rc=$?
  tail -1 $O/suite.log; grep -E "^FAILED|^ERROR" $O/suite.log | head -20
  exit $rc ;;
suites)
  O=gpurun_out/r06suite; mkdir -p $O
  for F in default ${1:-2 1 0}; do
    if [ $F = default ]; then E=""; else E="GI_X_WF=$F"; fi
    env $E timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite_$F.log 2>&1; rc=$?
    echo "suite $F: $(tail -1 $O/suite_$F.log)"
    [ $rc -eq 0 ] || { grep -E "^FAILED|Error" $O/suite_$F.log | head -5; exit 1; }
  done ;;
formab)
  O=gpurun_out/r06form; mkdir -p $O
  WL=${1//,/ }; shift
  for SPEC in "$@"; do
    V=${SPEC%%:*}; E=""; [[ "$SPEC" == *:* ]] && E=${SPEC#*:}; E=${E//,/ }
    T=${V}_$(echo "$E" | tr ' =' '_-')
    env GI_LIB=$(lib $V) $E timeout -k 10 400 python3 -u profiles/wf_probe.py --steps 3 --warmup 1 --forms ${FORMS:-mega,wf,seg} $WL > $O/$T.jsonl 2> $O/$T.err || { echo "FAIL $SPEC"; tail -5 $O/$T.err; exit 1; }
    python3 - "$O/$T.jsonl" "$SPEC" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    f = " ".join("%s %8.3f" % (k, d[k]["pass_ms"]) for k in ("mega", "wf", "seg") if k in d)
    print("%-30s %-11s %s  identical %s" % (sys.argv[2], d["workload"], f, d.get("identical")), flush=True)
PY
  done ;;
rab)
  O=gpurun_out/r06rab; mkdir -p $O
  for SPEC in "$@"; do
    V=${SPEC%%:*}; E=""; [[ "$SPEC" == *:* ]] && E=${SPEC#*:}; E=${E//,/ }
    T=${V}_$(echo "$E" | tr ' =' '_-')
    env GI_LIB=$(lib $V) $E timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
      -k "soup100k or mode_r_vs_reference_golden or split or candidate_reconstruction or mode_r_entities or mode_r_random" > $O/parity_$T.log 2>&1 || { echo "PARITY FAIL $SPEC"; tail -15 $O/parity_$T.log; exit 1; }
    echo "parity ok $SPEC: $(tail -1 $O/parity_$T.log)"
    for W in R-C4 R-C3; do
      env GI_LIB=$(lib $V) $E timeout -k 10 200 python3 bench.py --workload $W --steps 5 --warmup 1 --no-cpu-baseline --no-host-path > $O/${W}_$T.json 2> $O/${W}_$T.err || { echo "bench fail $SPEC $W"; tail -5 $O/${W}_$T.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${W}_$T.json').read().strip().splitlines()[-1]); print('%-30s %-6s kernel %.4f ms  frame %.4f ms' % ('$SPEC', '$W', d['roofline']['kernel_ms'], d['ms_per_step']))"
    done
  done ;;
benchq)
  O=gpurun_out/r06bq; mkdir -p $O
  for W in ${1//,/ }; do
    timeout -k 10 200 python3 bench.py --workload $W --steps ${2:-5} --warmup 1 --no-cpu-baseline --no-host-path > $O/bench_$W.json 2> $O/bench_$W.err || { echo "bench $W failed"; tail -5 $O/bench_$W.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_$W.json').read().strip().splitlines()[-1]); print('$W', d['roofline']['kernel'], d['roofline']['kernel_ms'], d['ms_per_step'], d['value'], json.dumps(d.get('schedule')))"
  done ;;
ab)
  O=gpurun_out/r06ab; mkdir -p $O
  WL=${1//,/ }; shift
  for REP in 1 2; do
  for SPEC in "$@"; do
    V=${SPEC%%:*}; E=""; [[ "$SPEC" == *:* ]] && E=${SPEC#*:}; E=${E//,/ }
    T=${V}_$(echo "$E" | tr ' =' '_-')
    for W in $WL; do
      env GI_LIB=$(lib $V) $E timeout -k 10 200 python3 bench.py --workload $W --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-host-path > $O/${W}_$T.json 2> $O/${W}_$T.err || { echo "bench fail $SPEC $W"; tail -5 $O/${W}_$T.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${W}_$T.json').read().strip().splitlines()[-1]); print('%-34s %-6s kernel %.4f ms  frame %.4f ms' % ('$SPEC', '$W', d['roofline']['kernel_ms'], d['ms_per_step']))"
    done
  done
  done ;;
ktrace)
  O=$GRAFT_REPO_ROOT/gpurun_out/r06kt; mkdir -p $O
  WL=${1//,/ }; shift
  export TMPDIR=/tmp
  for SPEC in "$@"; do
    V=${SPEC%%:*}; E=""; [[ "$SPEC" == *:* ]] && E=${SPEC#*:}; E=${E//,/ }
    T=${V}_$(echo "$E" | tr ' =' '_-')
    for W in $WL; do
      D=$O/${W}_$T
      ( cd /tmp && env GI_LIB=$(lib $V) $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload $W --steps 5 --warmup 1 --no-cpu-baseline --no-host-path > $D.log 2>&1 ) || { echo "ktrace fail $SPEC $W"; tail -5 $D.log; exit 1; }
      python3 - "$D" "$SPEC" "$W" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("void gi::(anonymous namespace)::", "").replace("gi::(anonymous namespace)::", "").split("(gi::")[0]
    if float(r["TotalDurationNs"]) > 20000:
        print("%-26s %-6s %-60s calls %4d  avg %9.1f us" % (sys.argv[2], sys.argv[3], n[:60], int(r["Calls"]), float(r["AverageNs"]) / 1e3))
PY
    done
  done ;;
tk)
  O=gpurun_out/r06tk; mkdir -p $O
  timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$1" > $O/tests.log 2>&1 || { grep -E "FAILED|Error|error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
  if [ -n "$2" ]; then bash $0 benchq $2; fi
  ;;
mem)
  # memory-pipeline counters (L2 read latency seen by the L1, TA / TCP stalls, instruction cache)
  # of a workload's dominant kernel per spec: gpurun_out/r06mem/<w>_mem_<variant>.json
  O=gpurun_out/r06mem; mkdir -p $O
  WL=${1//,/ }; shift
  for SPEC in "$@"; do
    V=${SPEC%%:*}; E=""; [[ "$SPEC" == *:* ]] && E=${SPEC#*:}; E=${E//,/ }
    for W in $WL; do
      w=$(echo $W | tr A-Z a-z); T=${w}_mem_${V}
      env GI_LIB=$(lib $V) $E PMC_PASSES="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCP_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum;TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum;SQC_ICACHE_MISSES SQC_ICACHE_HITS GRBM_GUI_ACTIVE;TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_LFIFO_STALL_CYCLES_sum;SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
        timeout -k 10 900 bash profiles/run_profile.sh $T --workload $W --steps 3 --warmup 1 > $O/$T.log 2>&1 || { echo "mem $SPEC $W failed"; tail -5 $O/$T.log; exit 1; }
      python3 profiles/summarize.py gpurun_out/prof_$T $W auto $O/$T.json 4 > /dev/null || exit 1
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['counters_per_launch']; print(sys.argv[2], sys.argv[3], round(d['avg_launch_ns']/1e6,4), {k: round(v) for k, v in sorted(c.items())})" $O/$T.json $SPEC $W
    done
  done ;;
evidence)
  O=gpurun_out/r06ev; mkdir -p $O
  case $1 in
  1)
    timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -20 $O/gpu_tests.log; exit 1; }
    tail -1 $O/gpu_tests.log
    timeout -k 10 1000 bash profiles/profile.sh r06 ${WLS:-C3 C2 C4 R-C4 C5} > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; } ;;
  2)
    for W in R-C4 C3 C4 C5; do
      timeout -k 10 300 python3 profiles/shard_scaling.py --workload $W > $O/shard_$W.jsonl 2>&1 || { tail -5 $O/shard_$W.jsonl; exit 1; }
      tail -1 $O/shard_$W.jsonl | cut -c1-300
    done
    for W in C2 C4 C5 R-C4 R-C3 R-main X-main X-zoo X-soup1000; do
      timeout -k 10 300 python3 bench.py --workload $W --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_$W.json 2> $O/bench_$W.err || { tail -5 $O/bench_$W.err; exit 1; }
    done
    timeout -k 10 300 python3 bench.py --workload C3 --steps 20 --warmup 2 > $O/bench_C3.json 2> $O/bench_C3.err || { tail -5 $O/bench_C3.err; exit 1; }
    timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --dist-backend gloo --workload C3 --steps 3 --warmup 1 > $O/rehearsal_n8_gloo.log 2>&1 || { tail -20 $O/rehearsal_n8_gloo.log; exit 1; }
    tail -1 $O/rehearsal_n8_gloo.log | cut -c1-300 ;;
  forms)
    GI_X_WF=0 timeout -k 10 600 bash profiles/profile.sh r06mega C3 > $O/prof_mega.log 2>&1 || { tail -5 $O/prof_mega.log; exit 1; }
    GI_X_WF=1 timeout -k 10 900 bash profiles/profile.sh r06wf C3 C5 > $O/prof_wf.log 2>&1 || { tail -5 $O/prof_wf.log; exit 1; }
    GI_X_WF=2 timeout -k 10 600 bash profiles/profile.sh r06seg C5 > $O/prof_seg.log 2>&1 || { tail -5 $O/prof_seg.log; exit 1; } ;;
  esac
  echo "evidence $1 done" ;;
final)
  # round-6 final evidence: suite; PMC of the Mode R workloads (their kernels changed after evidence 1);
  # a rocprofv3 kernel trace of the default C3 bench itself (the line and the trace from one process);
  # bench lines of R-C4 / R-C3 against the fresh PMC, and the default C3 bench with its CPU baseline
  O=gpurun_out/r06fin; mkdir -p $O
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -20 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
  timeout -k 10 900 bash profiles/profile.sh r06 R-C4 R-C3 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
  cp gpurun_out/r06prof/r06_r-c4_pmc.json gpurun_out/r06prof/r06_r-c3_pmc.json profiles/
  export TMPDIR=/tmp
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/c3trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-host-path > $GRAFT_REPO_ROOT/$O/C3_under_rocprof.json 2> $GRAFT_REPO_ROOT/$O/C3_under_rocprof.err ) || { tail -5 $O/C3_under_rocprof.err; exit 1; }
  for W in R-C4 R-C3; do
    timeout -k 10 300 python3 bench.py --workload $W --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_$W.json 2> $O/bench_$W.err || { tail -5 $O/bench_$W.err; exit 1; }
  done
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 2 > $O/bench_C3.json 2> $O/bench_C3.err || { tail -5 $O/bench_C3.err; exit 1; }
  tail -c 300 $O/bench_C3.json
  echo "final done" ;;
*)
  sed -n 2,19p "$0"; exit 2 ;;
esac
