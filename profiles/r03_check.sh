#!/bin/bash
# round 3: GPU suite (tag $1), then bench lines for the workloads given after it
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=$1; shift
bash profiles/gpu_tests.sh $TAG || exit 1
[ $# -gt 0 ] && bash profiles/benchall.sh "$@"
