#!/bin/bash
# A/B of the spatial-split BVH build (GI_XSBVH=1) on the 100k soup: Mode X parity with the knob
# on, then C4/C5 kernel time default vs SBVH
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
GI_XSBVH=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_mode_x_mirror.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -k "mode_x or sharded or mirror" > gpurun_out/sbvh_t.log 2>&1 \
  || { echo "PARITY FAIL sbvh"; tail -5 gpurun_out/sbvh_t.log; exit 1; }
echo "parity ok sbvh: $(tail -1 gpurun_out/sbvh_t.log)"
bash profiles/abx.sh C4,C5 default default:GI_XSBVH=1 default default:GI_XSBVH=1
