#!/bin/bash
# round 4: quick bench lines (no CPU baseline / host path) with kernel ms and the schedule block
#   profiles/r04_benchq.sh <workloads, comma> [steps]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04bq; mkdir -p $O
for W in ${1//,/ }; do
  timeout -k 10 200 python3 bench.py --workload $W --steps ${2:-5} --warmup 1 --no-cpu-baseline --no-host-path > $O/bench_$W.json 2> $O/bench_$W.err || { echo "bench $W failed"; tail -5 $O/bench_$W.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$W.json').read().strip().splitlines()[-1]); print('$W', d['roofline']['kernel'], d['roofline']['kernel_ms'], d['ms_per_step'], d['value'], json.dumps(d.get('schedule')))"
done
