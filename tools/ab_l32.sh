#!/bin/bash
# A/B of the 4-wave solvers: 32-bit lattice keys (sap_solve_mw_l32, default)
# vs round 2's 64-bit scaled keys (SH_FLAG_SP2 = 2048): one GPU's shard of a
# round at 8 GPUs (466 blocks, LDS tile) and 4 GPUs (933, register tile), at
# rounds 0 and 10, and the lone first block of round 0 (LDS tile, flag 8).
cd "$(dirname "$0")/.." || exit 2
out=${1:-gpurun_out/ab_l32.jsonl}
: > "$out"
for rep in 1 2; do
  for fl in 0 2048; do
    for B in 466 933; do
      for sr in 0 10; do
        timeout -k 10 120 python -u tools/probe.py --phase solve --reps 3 --blocks $B --flags $fl --state-round $sr \
          | tail -1 | sed "s/^/{\"flags\": $fl, \"blocks\": $B, \"state_round\": $sr, \"r\": /; s/$/}/" >> "$out" || exit 1
      done
    done
    timeout -k 10 120 python -u tools/probe.py --phase solve --reps 3 --blocks 1 --flags $((fl | 8)) \
      | tail -1 | sed "s/^/{\"flags\": $((fl | 8)), \"lone\": 1, \"r\": /; s/$/}/" >> "$out" || exit 1
  done
done
python3 - "$out" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    x = json.loads(l)
    d[(x["flags"], x.get("blocks", 1), x.get("state_round", 0))].append(x["r"]["solve"]["ms"])
for k, v in sorted(d.items()):
    print(k, min(v))
PY
