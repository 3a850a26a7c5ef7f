#!/bin/bash
# round-4 GPU session 25: santa_dt_kernel's per-Dijkstra dual update with the
# LDS atomics and path-row reads of the visited columns only (exec-masked)
# instead of every lane (a dump slot for the others): abl/dv1 vs abl/dv0
cd /root/repo
bash tools/ab_libs.sh gpurun_out/ab_r4y.jsonl "--blocks 466 --phase solve --reps 3" \
  "--blocks 466 --phase solve --reps 3 --state-round 10" "--blocks 1 --flags 4096 --phase solve --reps 3" \
  -- abl/dv0.so abl/dv1.so > gpurun_out/ab_r4y.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab_r4y.log | cut -c1-110
echo all-done
