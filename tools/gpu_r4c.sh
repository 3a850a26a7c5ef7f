#!/bin/bash
# round-4 GPU session 3: the suite on the key-unit sparse step (sbp = value |
# step, indexed book-keeping), then an A/B of abl/r4f.so (fused build, round-4
# step) against abl/r4g.so (key-unit step)
cd /root/repo
bash tools/gpu_run.sh tests smoke bench || exit 1
bash tools/ab_libs.sh gpurun_out/ab_r4g.jsonl \
  "--phase solve --reps 3" "--phase solve --reps 3 --state-round 10" \
  "--blocks 1 --flags 128 --phase solve --reps 3" "--blocks 1865 --phase solve --reps 3" \
  -- abl/r4f.so abl/r4g.so > gpurun_out/ab_r4g.log 2>&1 || exit 1
echo all-done
