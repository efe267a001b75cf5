set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04a
timeout -k 10 200 python3 bench.py --workload C3 --steps 10 --warmup 2 --no-cpu-baseline --no-host-path > gpurun_out/r04a/c3.json 2>gpurun_out/r04a/c3.err &&
timeout -k 10 600 bash profiles/profile.sh r04 C2 > gpurun_out/r04a/prof.log 2>&1 &&
timeout -k 10 200 python3 bench.py --workload C2 --steps 20 --warmup 2 --no-cpu-baseline --no-host-path > gpurun_out/r04a/c2.json 2>gpurun_out/r04a/c2.err
echo rc=$?
