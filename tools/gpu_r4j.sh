#!/bin/bash
# round-4 GPU session 10: parity on the sparse step's trimmed entry decode
# (bit-field offsets i << 4) and stepped `remaining` address; A/B of abl/r4o.so
# (profiled source) against abl/r4p.so and abl/r4q.so (r4p + issue-priority
# thresholds 48 / 12 / 3 instead of 32 / 8 / 2)
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "bench_rounds or round_vs_oracle or designs_agree or edge_block or small_wishlists or sparse_overflow" \
  > gpurun_out/tests_r4p.log 2>&1 || { tail -30 gpurun_out/tests_r4p.log; exit 1; }
tail -2 gpurun_out/tests_r4p.log
bash tools/ab_libs.sh gpurun_out/ab_r4p.jsonl \
  "--phase solve --reps 3" "--phase solve --reps 3 --state-round 10" \
  "--blocks 1 --flags 128 --phase solve --reps 3" "--blocks 933 --phase solve --reps 3" \
  -- abl/r4o.so abl/r4p.so abl/r4q.so > gpurun_out/ab_r4p.log 2>&1 || exit 1
echo all-done
