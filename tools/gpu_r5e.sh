#!/bin/bash
# round-5 GPU session: santa_lb_kernel variants (second-best prefetch on/off,
# packed/int16 rows): parity subset per variant, then A/B probes
cd /root/repo
for v in lb_pf1_pk1 lb_pf0_pk1 lb_pf0_pk0 lb_pf1_pk0; do
  SANTA_HIP_LIB=abl/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread \
    -k "reference_sizes or round_vs_oracle or wave_configs" > gpurun_out/r5e_tests_$v.log 2>&1 || { echo "FAIL $v"; tail -30 gpurun_out/r5e_tests_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r5e_tests_$v.log)"
done
bash tools/ab_libs.sh gpurun_out/r5e_ab.jsonl "--n 2000 --blocks 1 --phase solve --reps 3" "--n 2000 --phase solve --reps 2" \
  "--n 2000 --phase solve --reps 2 --state-round 10" -- abl/lb_pf1_pk1.so abl/lb_pf0_pk1.so abl/lb_pf0_pk0.so abl/lb_pf1_pk0.so \
  > gpurun_out/r5e_ab.log 2>&1 || { tail -20 gpurun_out/r5e_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5e_ab.log | cut -c1-120
SANTA_HIP_LIB=abl/lb_pf0_pk1.so bash tools/gpu_r5c.sh
echo all-done
