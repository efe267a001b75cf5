# Round-6 final evidence after the own-plane skip (Mode X) and the reach lane groups (Mode R):
# PMC + kernel stats of C3 C2 R-C4 C4 R-C3; the same-process rocprofv3 trace of the default C3 bench;
# shard probes, bench lines of every workload, the C3 bench with its CPU baseline, the 8-rank gloo rehearsal
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06fin2
O=gpurun_out/r06fin2
timeout -k 10 1000 bash profiles/profile.sh r06 C3 C2 R-C4 C4 R-C3 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
echo "pmc done"
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/c3trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-host-path > $GRAFT_REPO_ROOT/$O/C3_under_rocprof.json 2> $GRAFT_REPO_ROOT/$O/C3_under_rocprof.err ) || { tail -5 $O/C3_under_rocprof.err; exit 1; }
echo "trace done"
timeout -k 10 1200 bash profiles/r06.sh evidence 2 || exit 1
