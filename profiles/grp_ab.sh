set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/grp
for v in g4 g2 g8; do
  GI_LIB=$PWD/2019global_amd/_variants/libgi_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread -k "c4_config or c5_config or forms_bit_identical or soup100k_full" > gpurun_out/grp/t_$v.log 2>&1 || { echo "FAIL $v"; grep -E "FAILED|Error|assert" gpurun_out/grp/t_$v.log | head; tail -5 gpurun_out/grp/t_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/grp/t_$v.log)"
done
bash profiles/r05.sh ab C4 default g4 g2 g8
