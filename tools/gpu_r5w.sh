#!/bin/bash
# round-5 GPU session: santa_dt_kernel (the 8-GPU shard kernel) with
# santa_sp3_kernel's SALU -> VALU step: parity, A/B against HEAD
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "designs_agree or round_vs_oracle or shard or dense or argmin_agree or solve_round" \
  > gpurun_out/r5w_tests.log 2>&1 || { grep -E "Error|error|assert|FAIL" gpurun_out/r5w_tests.log | head -30; exit 1; }
tail -1 gpurun_out/r5w_tests.log
bash tools/ab_libs.sh gpurun_out/r5w_ab.jsonl \
  "--blocks 466 --phase solve --reps 5" "--blocks 466 --phase solve --reps 5 --state-round 10" "--blocks 1 --flags 4096 --phase solve --reps 5" \
  -- abl/libsanta_hip_a.so abl/libsanta_hip_b.so > gpurun_out/r5w_ab.log 2>&1 || { tail gpurun_out/r5w_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5w_ab.log | cut -c1-160
echo all-done
