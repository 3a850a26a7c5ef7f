#!/bin/bash
# round-4 GPU session 9: the dense-tile kernel's fast build (packed
# wishlists, one row per thread) -- parity, then A/B of abl/r4n0.so (chain
# build) against abl/r4n.so (fast build) on the 8-GPU shard and a lone block,
# and of abl/r4n.so against abl/r4o.so (the same fast build in the 4-wave
# twins kernel) on twins rounds
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "round_vs_oracle or designs_agree or edge_block or argmin_agree or no_apply or out_of_range or dispatch or small_wishlists or shard" \
  > gpurun_out/tests_r4n.log 2>&1 || { tail -30 gpurun_out/tests_r4n.log; exit 1; }
tail -2 gpurun_out/tests_r4n.log
bash tools/ab_libs.sh gpurun_out/ab_r4n.jsonl \
  "--blocks 466 --phase solve --reps 3" "--blocks 466 --phase solve --reps 3 --state-round 10" \
  "--blocks 466 --phase build --reps 3" "--blocks 1 --flags 4096 --phase solve --reps 3" \
  -- abl/r4n0.so abl/r4n.so > gpurun_out/ab_r4n.log 2>&1 || exit 1
bash tools/ab_libs.sh gpurun_out/ab_r4o.jsonl \
  "--mode 1 --phase solve --reps 3" "--mode 1 --phase solve --reps 3 --state-round 10" \
  "--mode 1 --phase build --reps 3" "--mode 1 --blocks 1 --phase solve --reps 3" \
  -- abl/r4n.so abl/r4o.so > gpurun_out/ab_r4o.log 2>&1 || exit 1
echo all-done
