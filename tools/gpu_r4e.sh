#!/bin/bash
# round-4 GPU session 4: parity on the per-Dijkstra trims (tie-bit table, sink-only assignment mask, indexed path select, bounded augmentation), A/B of
# abl/r4g.so against abl/r4i.so, the fused build alone, and the step segments
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "bench_rounds or round_vs_oracle or designs_agree or sparse_overflow or edge_block or argmin_agree" \
  > gpurun_out/tests_r4i.log 2>&1 || { tail -30 gpurun_out/tests_r4i.log; exit 1; }
tail -2 gpurun_out/tests_r4i.log
bash tools/ab_libs.sh gpurun_out/ab_r4i.jsonl \
  "--phase solve --reps 3" "--phase solve --reps 3 --state-round 10" \
  "--blocks 1 --flags 128 --phase solve --reps 3" "--phase build --reps 3" "--phase build --reps 3 --state-round 10" \
  -- abl/r4g.so abl/r4i.so > gpurun_out/ab_r4i.log 2>&1 || exit 1
for A in "--blocks 1 --flags 128 --phase solve --reps 1 --segments" "--phase solve --reps 1 --segments --state-round 10"; do
  timeout -k 10 300 python -u tools/probe.py $A >> gpurun_out/seg_r4i.jsonl 2>/dev/null || exit 1
done
echo all-done
