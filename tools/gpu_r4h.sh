#!/bin/bash
# round-4 GPU session 8: the whole GPU suite with the dense-tile kernels as the
# few-block default; A/B of abl/r4m1.so (dense-tile stores by one lane) against
# abl/r4m.so (by all lanes, as the sparse kernel); twins on the one-wave
# dense-tile kernel (SH_FLAG_DT_TILE) against the 4-wave LDS tile
cd /root/repo
bash tools/gpu_run.sh tests smoke || exit 1
grep -q " passed" gpurun_out/tests.log && ! grep -q " failed" gpurun_out/tests.log || exit 1
bash tools/ab_libs.sh gpurun_out/ab_r4m.jsonl \
  "--blocks 466 --phase solve --reps 3" "--blocks 466 --phase solve --reps 3 --state-round 10" \
  "--blocks 1 --flags 4096 --phase solve --reps 3" "--phase solve --reps 3 --state-round 10" \
  "--mode 1 --flags 4096 --phase solve --reps 3" "--mode 1 --blocks 1 --flags 4096 --phase solve --reps 3" \
  -- abl/r4m1.so abl/r4m.so > gpurun_out/ab_r4m.log 2>&1 || exit 1
for A in "--mode 1" "--mode 1 --flags 4096" "--mode 1 --state-round 10" "--mode 1 --flags 4096 --state-round 10" \
         "--mode 1 --blocks 1" "--mode 1 --blocks 1 --flags 4096" "--blocks 933" "--blocks 933 --flags 32"; do
  r=$(timeout -k 10 120 python tools/probe.py --phase solve --reps 3 $A) || exit 1
  echo "{\"args\": \"$A\", \"r\": $r}" >> gpurun_out/twins_dt.jsonl
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_r4m.json 2> gpurun_out/bench_r4m.err || exit 1
timeout -k 10 300 python -u bench.py --mode twins --no-cpu-baseline > gpurun_out/bench_r4m_twins.json 2> gpurun_out/bench_r4m_twins.err || exit 1
echo all-done
