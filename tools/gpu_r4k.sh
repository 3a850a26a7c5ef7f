#!/bin/bash
# round-4 GPU session 11: parity with the tie-bit table flipped per sink and
# the precomputed `remaining` (sparse and dense-tile kernels); A/B of
# abl/r4p.so against abl/r4r.so
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "bench_rounds or round_vs_oracle or designs_agree or edge_block or small_wishlists or sparse_overflow or declines or shard" \
  > gpurun_out/tests_r4r.log 2>&1 || { tail -30 gpurun_out/tests_r4r.log; exit 1; }
tail -2 gpurun_out/tests_r4r.log
bash tools/ab_libs.sh gpurun_out/ab_r4r.jsonl \
  "--phase solve --reps 3" "--phase solve --reps 3 --state-round 10" "--blocks 1 --flags 128 --phase solve --reps 3" \
  "--blocks 466 --phase solve --reps 3" "--blocks 466 --phase solve --reps 3 --state-round 10" \
  "--blocks 1 --flags 4096 --phase solve --reps 3" \
  -- abl/r4p.so abl/r4r.so > gpurun_out/ab_r4r.log 2>&1 || exit 1
echo all-done
