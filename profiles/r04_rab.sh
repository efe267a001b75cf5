#!/bin/bash
# round 4: Mode R A/B over kernel variants -- parity of the Mode R frames (goldens, reverse-DFS
# equality incl. the whole 100k-soup frame), then R-C4 / R-C3 bench lines
#   profiles/r04_rab.sh <variant>[:ENV=v,...] ...   (variant "default" = libgi.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04rab; mkdir -p $O
for SPEC in "$@"; do
  V=${SPEC%%:*}; E=""; [[ "$SPEC" == *:* ]] && E=${SPEC#*:}; E=${E//,/ }
  if [ "$V" = default ]; then LIB=$GRAFT_REPO_ROOT/2019global_amd/libgi.so; else LIB=$GRAFT_REPO_ROOT/2019global_amd/_variants/libgi_$V.so; fi
  T=${V}_$(echo "$E" | tr ' =' '_-')
  env GI_LIB=$LIB $E timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "soup100k or mode_r_vs_reference_golden or split or candidate_reconstruction or mode_r_entities or mode_r_random" > $O/parity_$T.log 2>&1 || { echo "PARITY FAIL $SPEC"; tail -15 $O/parity_$T.log; exit 1; }
  echo "parity ok $SPEC: $(tail -1 $O/parity_$T.log)"
  for W in R-C4 R-C3; do
    env GI_LIB=$LIB $E timeout -k 10 200 python3 bench.py --workload $W --steps 5 --warmup 1 --no-cpu-baseline --no-host-path > $O/${W}_$T.json 2> $O/${W}_$T.err || { echo "bench fail $SPEC $W"; tail -5 $O/${W}_$T.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/${W}_$T.json').read().strip().splitlines()[-1]); print('%-30s %-6s kernel %.4f ms  frame %.4f ms' % ('$SPEC', '$W', d['roofline']['kernel_ms'], d['ms_per_step']))"
  done
done
