#!/bin/bash
# round-4 GPU session: tests, smoke, bench lines; then an A/B of abl/base.so
# (round 3's kernels minus santa_sp2_kernel) against abl/r4b.so (the tree)
cd /root/repo
bash tools/gpu_run.sh tests smoke bench bench_twins || exit 1
bash tools/ab_libs.sh gpurun_out/ab_r4b.jsonl \
  "--blocks 1 --flags 128 --phase solve --reps 3" "--phase solve --reps 3" \
  "--phase solve --reps 3 --state-round 10" "--blocks 1 --flags 8 --phase solve --reps 3" \
  "--blocks 466 --phase solve --reps 3" "--mode 1 --phase solve --reps 3" \
  "--mode 1 --blocks 1 --phase solve --reps 3" -- abl/base.so abl/r4b.so > gpurun_out/ab_r4b.log 2>&1 || exit 1
echo all-done
