#!/bin/bash
# round-4 GPU session 7: A/B of abl/r4i.so against abl/r4k.so (pass-2 writes
# without per-wish tests) and abl/r4l.so (+ single-lane same-word stores in
# the step); then the N = 8 / N = 4 shards on the one-wave sparse kernel
# (SH_FLAG_SP_TILE = 128) and the dense-tile one-wave kernel (SH_FLAG_DT_TILE =
# 4096) against their default 4-wave designs (in-tree library)
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "bench_rounds or round_vs_oracle or sparse_overflow or small_wishlists or designs_agree or edge_block or argmin_agree or no_apply or out_of_range or dispatch" \
  > gpurun_out/tests_r4l.log 2>&1 || { tail -30 gpurun_out/tests_r4l.log; exit 1; }
tail -2 gpurun_out/tests_r4l.log
bash tools/ab_libs.sh gpurun_out/ab_r4k.jsonl \
  "--phase solve --reps 3" "--phase solve --reps 3 --state-round 10" \
  "--blocks 1 --flags 128 --phase solve --reps 3" "--blocks 1865 --phase solve --reps 3" \
  -- abl/r4i.so abl/r4k.so abl/r4l.so > gpurun_out/ab_r4k.log 2>&1 || exit 1
for A in "--blocks 466" "--blocks 466 --flags 128" "--blocks 466 --flags 4096" \
         "--blocks 466 --state-round 10" "--blocks 466 --flags 128 --state-round 10" "--blocks 466 --flags 4096 --state-round 10" \
         "--blocks 933" "--blocks 933 --flags 128" "--blocks 933 --flags 4096" \
         "--blocks 1 --flags 8" "--blocks 1 --flags 4096" "--blocks 1 --flags 128"; do
  r=$(timeout -k 10 120 python tools/probe.py --phase solve --reps 3 $A) || exit 1
  echo "{\"args\": \"$A\", \"r\": $r}" >> gpurun_out/shard_sp3_r4l.jsonl
done
echo all-done
