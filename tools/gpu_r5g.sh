#!/bin/bash
# round-5 GPU session: santa_lb_kernel wave/column splits at n = 2000
# (8 x 4, 4 x 8, 16 x 2): parity subset per variant, then A/B probes
cd /root/repo
for v in lb_c2; do
  SANTA_HIP_LIB=abl/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread \
    -k "reference_sizes or round_vs_oracle or wave_configs" > gpurun_out/r5g_tests_$v.log 2>&1 || { echo "FAIL $v"; tail -30 gpurun_out/r5g_tests_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r5g_tests_$v.log)"
done
bash tools/ab_libs.sh gpurun_out/r5g_ab.jsonl "--n 2000 --blocks 1 --phase solve --reps 3" "--n 2000 --phase solve --reps 2" \
  "--n 2000 --phase solve --reps 2 --state-round 10" -- abl/lb_c0.so abl/lb_c1.so abl/lb_c2.so \
  > gpurun_out/r5g_ab.log 2>&1 || { tail -20 gpurun_out/r5g_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5g_ab.log | cut -c1-120
SANTA_HIP_LIB=abl/lb_c0.so bash tools/gpu_r5c.sh
echo all-done
