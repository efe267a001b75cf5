#!/bin/bash
# Mode R: ImpTriangle-only specialisation of k_mode_r_split (default) vs none (notri) vs axis-by-axis
# line node test (rax): Mode R GPU parity subset per variant, then R-C4 kernel time, twice
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for V in default notri rax; do
  if [ "$V" = default ]; then LIB=$R/2019global_amd/libgi.so; else LIB=$R/2019global_amd/_variants/libgi_$V.so; fi
  GI_LIB=$LIB timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "mode_r or split_candidates or raytracer_api or expbox or trace_ray" > gpurun_out/rt_t_$V.log 2>&1 || { echo "PARITY FAIL $V"; tail -5 gpurun_out/rt_t_$V.log; exit 1; }
  echo "parity ok $V: $(tail -1 gpurun_out/rt_t_$V.log)"
done
for rep in 1 2; do for V in default notri rax; do
  if [ "$V" = default ]; then LIB=$R/2019global_amd/libgi.so; else LIB=$R/2019global_amd/_variants/libgi_$V.so; fi
  GI_LIB=$LIB timeout -k 10 300 python bench.py --workload R-C4 --steps 5 --warmup 2 --no-cpu-baseline --no-host-path > gpurun_out/rt_$V.log 2>&1 || { tail -5 gpurun_out/rt_$V.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/rt_$V.log').read().strip().splitlines()[-1]); print('$V R-C4 kern_ms', d['roofline']['kernel_ms'], 'ms', d['ms_per_step'])"
done; done
