#!/bin/bash
# round 4 evidence, part B: the forced-form profiles (C3 under k_mode_x and the wavefront form, C5
# under the wavefront and segment forms), bench lines, and the N = 8 gloo rehearsal on one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04ev; mkdir -p $O
GI_X_WF=0 timeout -k 10 600 bash profiles/profile.sh r04mega C3 > $O/prof_mega.log 2>&1 || { tail -5 $O/prof_mega.log; exit 1; }
GI_X_WF=1 timeout -k 10 900 bash profiles/profile.sh r04wf C3 C5 > $O/prof_wf.log 2>&1 || { tail -5 $O/prof_wf.log; exit 1; }
GI_X_WF=2 timeout -k 10 600 bash profiles/profile.sh r04seg C5 > $O/prof_seg.log 2>&1 || { tail -5 $O/prof_seg.log; exit 1; }
echo profiles done
for W in C2 C4 C5 R-C4 R-C3 X-main X-zoo X-soup1000; do
  timeout -k 10 300 python3 bench.py --workload $W --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_$W.json 2> $O/bench_$W.err || { tail -5 $O/bench_$W.err; exit 1; }
done
timeout -k 10 300 python3 bench.py --workload C3 --steps 20 --warmup 2 > $O/bench_C3.json 2> $O/bench_C3.err || { tail -5 $O/bench_C3.err; exit 1; }
echo benches done
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --dist-backend gloo --workload C3 --steps 3 --warmup 1 > $O/rehearsal_n8_gloo.log 2>&1 || { tail -20 $O/rehearsal_n8_gloo.log; exit 1; }
tail -1 $O/rehearsal_n8_gloo.log | cut -c1-300
echo evidence B done
