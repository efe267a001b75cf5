set -o pipefail
cd $GRAFT_REPO_ROOT
for v in k32 k16 k8; do
  GI_LIB=$PWD/2019global_amd/_variants/libgi_$v.so timeout -k 10 200 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread -k "soup100k or mode_r_kernels_frame or whole_frame" > gpurun_out/t_$v.log 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/t_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/t_$v.log)"
  GI_LIB=$PWD/2019global_amd/_variants/libgi_$v.so timeout -k 10 200 python3 profiles/shard_scaling.py --workload R-C4 --ns 1,8 | tail -1
done
bash profiles/r05.sh ab R-C4 default k32 k16 k8
