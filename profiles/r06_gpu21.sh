# After the Mode R acceptance fast path: whole GPU suite; PMC + kernel stats of R-C4 / R-C3; bench lines;
# the R-C4 share probe
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06fin4
O=gpurun_out/r06fin4
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; S=$?
tail -2 $O/gpu_tests.log; echo "suite rc $S"
if [ $S -ne 0 ]; then grep -E "^FAILED|^E " $O/gpu_tests.log | head -20; exit $S; fi
timeout -k 10 900 bash profiles/profile.sh r06 R-C4 R-C3 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
cp gpurun_out/r06prof/r06_r-c4_pmc.json gpurun_out/r06prof/r06_r-c3_pmc.json profiles/
for W in R-C4 R-C3 R-main; do
  timeout -k 10 300 python3 bench.py --workload $W --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_$W.json 2> $O/bench_$W.err || { tail -5 $O/bench_$W.err; exit 1; }
done
timeout -k 10 300 python3 profiles/shard_scaling.py --workload R-C4 > $O/shard_R-C4.jsonl 2>&1 || exit 1
tail -1 $O/shard_R-C4.jsonl | cut -c1-400
echo fin4 done
