#!/bin/bash
# GPU parity suite on the box: profiles/gpu_tests.sh <tag> [pytest -k expression]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-run}; shift
K=()
[ $# -gt 0 ] && K=(-k "$*")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread "${K[@]}" > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests_$TAG.log
exit $rc
