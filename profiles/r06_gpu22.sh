# C4 / C5 with other leaf sizes (GI_XLEAF_MAX test hook, read at scene build): kernel ms
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06leaf
for L in 2 4 8 6 4 2 8 4; do
  for W in C4; do
    GI_XLEAF_MAX=$L timeout -k 10 200 python3 bench.py --workload $W --steps 10 --warmup 2 --no-cpu-baseline --no-host-path > gpurun_out/r06leaf/${W}_$L.json 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/r06leaf/${W}_$L.json').read().strip().splitlines()[-1]); print('leaf $L $W kernel %.4f ms frame %.4f ms' % (d['roofline']['kernel_ms'], d['ms_per_step']))"
  done
done
