#!/bin/bash
# round-4 GPU session 19: the dense tile build with batched type-table reads
# and the twins code -> entry pass in 32-bit arithmetic (santa_dt_kernel,
# santa_block_kernel<1,1>): parity of the twins and dense-tile paths, then an
# A/B against the r04b library (abl/tw_base.so, the committed source)
cd /root/repo
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "santa_blocks_golden or round_vs_oracle or bench_rounds or designs_agree or edge_block or small_wishlists or declines or shard or reference_block_sizes or pipelined or full_round_properties" \
  > gpurun_out/tests_r4s.log 2>&1 || { tail -30 gpurun_out/tests_r4s.log; exit 1; }
tail -2 gpurun_out/tests_r4s.log
bash tools/ab_libs.sh gpurun_out/ab_r4s.jsonl \
  "--mode 1 --phase build --reps 5" "--mode 1 --phase solve --reps 3" "--mode 1 --phase solve --reps 3 --state-round 10" \
  "--blocks 466 --phase build --reps 5" "--blocks 466 --phase solve --reps 3" "--blocks 466 --phase solve --reps 3 --state-round 10" \
  -- abl/tw_base.so abl/tw_new.so > gpurun_out/ab_r4s.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab_r4s.log | cut -c1-110
echo all-done
