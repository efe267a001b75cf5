set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r02_s3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02_s3/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r02_s3/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r02_s3/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r02_s3/bench.json 2> gpurun_out/r02_s3/bench.err || { tail -5 gpurun_out/r02_s3/bench.err; exit 1; }
tail -1 gpurun_out/r02_s3/bench.json
bash profiles/r02_profile.sh C3 C4 R-C3 R-C4
