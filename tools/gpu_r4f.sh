#!/bin/bash
# round-4 GPU session 6: parity on the cheaper fused build (batch rows
# preloaded, first two columns written without per-wish tests), A/B of
# abl/r4i.so against abl/r4j.so
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "bench_rounds or round_vs_oracle or designs_agree or sparse_overflow or edge_block or argmin_agree or small_wishlists" \
  > gpurun_out/tests_r4j.log 2>&1 || { tail -30 gpurun_out/tests_r4j.log; exit 1; }
tail -2 gpurun_out/tests_r4j.log
bash tools/ab_libs.sh gpurun_out/ab_r4j.jsonl \
  "--phase solve --reps 3" "--phase solve --reps 3 --state-round 10" \
  "--phase build --reps 3" "--phase build --reps 3 --state-round 10" "--blocks 1865 --phase solve --reps 3" \
  -- abl/r4i.so abl/r4j.so > gpurun_out/ab_r4j.log 2>&1 || exit 1
echo all-done
