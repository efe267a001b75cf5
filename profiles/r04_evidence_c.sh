#!/bin/bash
# round 4 evidence at the final HEAD (k_mode_r_batch for Mode R, the classify pass's per-workgroup
# atomic): part 1 (PART=1) GPU suite + rocprofv3 stats/PMC of the default kernels; part 2 (PART=2)
# shard-scaling probes, bench lines of every workload, the C3 bench with its CPU baseline, and the
# N = 8 gloo rehearsal on one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04ev; mkdir -p $O
if [ "${PART:-1}" = 1 ]; then
  timeout -k 10 400 python3 -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -20 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
  timeout -k 10 1000 bash profiles/profile.sh r04 ${WLS:-C3 C2 C4 R-C4 C5} > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
  echo evidence part 1 done
else
  for W in R-C4 C3; do
    timeout -k 10 300 python3 profiles/shard_scaling.py --workload $W > $O/shard_$W.jsonl 2>&1 || { tail -5 $O/shard_$W.jsonl; exit 1; }
    tail -1 $O/shard_$W.jsonl | cut -c1-300
  done
  for W in C2 C4 C5 R-C4 R-C3 R-main X-main X-zoo X-soup1000; do
    timeout -k 10 300 python3 bench.py --workload $W --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_$W.json 2> $O/bench_$W.err || { tail -5 $O/bench_$W.err; exit 1; }
  done
  timeout -k 10 300 python3 bench.py --workload C3 --steps 20 --warmup 2 > $O/bench_C3.json 2> $O/bench_C3.err || { tail -5 $O/bench_C3.err; exit 1; }
  echo benches done
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --dist-backend gloo --workload C3 --steps 3 --warmup 1 > $O/rehearsal_n8_gloo.log 2>&1 || { tail -20 $O/rehearsal_n8_gloo.log; exit 1; }
  tail -1 $O/rehearsal_n8_gloo.log | cut -c1-300
  echo evidence part 2 done
fi
