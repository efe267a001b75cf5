#!/bin/bash
# round 4: Mode R heavy-pixel hand-off (GI_R_BUDGET) -- parity of the soup frames at two budgets,
# then R-C4 bench lines over a budget sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04rb; mkdir -p $O
for B in 8 48; do
  GI_R_BUDGET=$B timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "soup100k or mode_r_vs_reference_golden or split or candidate_reconstruction" > $O/parity_$B.log 2>&1 || { echo "parity FAIL budget $B"; tail -15 $O/parity_$B.log; exit 1; }
  echo "parity ok budget $B: $(tail -1 $O/parity_$B.log)"
done
for B in 0 8 16 32 64 128 256; do
  GI_R_BUDGET=$B timeout -k 10 200 python3 bench.py --workload R-C4 --steps 5 --warmup 1 --no-cpu-baseline --no-host-path > $O/rc4_$B.json 2> $O/rc4_$B.err || { echo "bench fail $B"; tail -5 $O/rc4_$B.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/rc4_$B.json').read().strip().splitlines()[-1]); print('budget $B', d['roofline']['kernel_ms'], d['ms_per_step'], d['roofline']['node_visits'], d['roofline']['prim_tests'])"
done
