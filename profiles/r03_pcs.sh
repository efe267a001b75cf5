#!/bin/bash
# PC sampling (rocprofv3, stochastic hardware sampling, cycles) of the C3 / C5 bench kernels on a
# line-table build of the library (_variants/libgi_dbg.so): where the k_mode_x cycles go
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/pcs
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/pcs/list.txt 2>&1; echo "list rc $?"
cd $R
W=${1:-C3}
GI_LIB=$R/2019global_amd/_variants/libgi_dbg.so timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled \
  --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 1048576 \
  -d gpurun_out/pcs/$W -o pcs --output-format csv -- python3 bench.py --workload $W --steps 2 --warmup 1 \
  --no-cpu-baseline --no-host-path > gpurun_out/pcs/run_$W.log 2>&1
echo "pcs rc $?"; tail -3 gpurun_out/pcs/run_$W.log; find gpurun_out/pcs -name "*.csv" | head
