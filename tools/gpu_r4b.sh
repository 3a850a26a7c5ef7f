#!/bin/bash
# round-4 GPU session 2: the suite on the fused in-kernel tile build, then an A/B
# of abl/r4c.so (tile kernel + record) against abl/r4f.so (fused)
cd /root/repo
bash tools/gpu_run.sh tests smoke bench || exit 1
bash tools/ab_libs.sh gpurun_out/ab_r4f.jsonl \
  "--phase solve --reps 3" "--phase solve --reps 3 --state-round 10" \
  "--blocks 1 --flags 128 --phase solve --reps 3" "--blocks 1865 --phase solve --reps 3" \
  -- abl/r4c.so abl/r4f.so > gpurun_out/ab_r4f.log 2>&1 || exit 1
for L in abl/r4c.so abl/r4f.so; do
  SANTA_HIP_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$(basename $L .so).json 2>gpurun_out/bench_$(basename $L .so).err || exit 1
done
echo all-done
