#!/bin/bash
# round-5 GPU session: santa_sp3_kernel's per-Dijkstra segment split (D0 set-up,
# D1 dual update, D2 augmentation) -- lone block, full round 0 and round 10
cd /root/repo
export TMPDIR=/tmp
for A in "--blocks 1 --flags 128 --phase solve --reps 1 --segments" "--phase solve --reps 1 --segments" \
         "--phase solve --reps 1 --segments --state-round 10" "--blocks 466 --phase solve --reps 1 --segments --state-round 10"; do
  timeout -k 10 300 python -u tools/probe.py $A >> gpurun_out/r5p_segments.jsonl 2>gpurun_out/r5p.err || { tail gpurun_out/r5p.err; exit 1; }
done
cut -c1-600 gpurun_out/r5p_segments.jsonl
echo all-done
