#!/bin/bash
# 4-wave solver latency probe: twins full round (78 blocks) at rounds 0/5,
# one GPU's 8-GPU shard (466 singles blocks, LDS tile) at rounds 0/10, and a
# lone block of each.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
P="timeout -k 10 120 python -u tools/probe.py --phase solve --reps 3"
{ $P --mode 1 && $P --mode 1 --state-round 5 && $P --blocks 466 && $P --blocks 466 --state-round 10 &&
  $P --mode 1 --blocks 1 && $P --blocks 1 --flags 8 && $P --blocks 3730 --state-round 10; } > gpurun_out/probe_w4.log 2>&1
rc=$?; grep '^{' gpurun_out/probe_w4.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); ms = d['solve']['ms']
    print(d['blocks'], d['state_round'], d['flags'], 'ms', round(ms, 4), 'steps_max', d['steps_max'], 'cyc/step(max blk @2.4GHz)', round(ms * 2.4e6 / d['steps_max']))
"; exit $rc
