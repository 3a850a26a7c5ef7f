#!/bin/bash
# quick state check: step segments (sp3 lone / full round 10; 4-wave LDS tile lone) and bench lines
cd "$(dirname "$0")/.." || exit 2
out=gpurun_out/quick.jsonl; : > $out
for args in "--blocks 1 --segments --phase solve --reps 1" "--segments --phase solve --reps 1 --state-round 10" \
            "--blocks 1 --flags 8 --segments --phase solve --reps 1"; do
  r=$(timeout -k 10 120 python tools/probe.py $args) || exit 1
  echo "{\"args\": \"$args\", \"r\": $r}" >> $out; echo "$args $(echo $r | cut -c1-400)"
done
for m in single twins; do
  timeout -k 10 300 python bench.py --mode $m --no-cpu-baseline > gpurun_out/quick_bench_$m.json || exit 1
  cut -c1-300 gpurun_out/quick_bench_$m.json
done
