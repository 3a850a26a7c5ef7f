#!/bin/bash
# A/B of the one-wave register-tile solvers on one box: santa_sp3_kernel
# (default, 32-bit lattice keys) vs santa_sp2_kernel (SH_FLAG_SP2 = 2048):
# full round 0 / round 10 (3730 blocks) and the lone longest block.
cd "$(dirname "$0")/.." || exit 2
out=${1:-gpurun_out/ab_sp3.jsonl}
: > "$out"
for rep in 1 2; do
  for fl in 0 2048; do
    for sr in 0 10; do
      timeout -k 10 120 python -u tools/probe.py --phase solve --reps 3 --flags $fl --state-round $sr \
        | tail -1 | sed "s/^/{\"flags\": $fl, \"state_round\": $sr, \"r\": /; s/$/}/" >> "$out" || exit 1
    done
    timeout -k 10 120 python -u tools/probe.py --phase solve --reps 3 --blocks 1 --flags $((fl | 128)) \
      | tail -1 | sed "s/^/{\"flags\": $((fl | 128)), \"lone\": 1, \"r\": /; s/$/}/" >> "$out" || exit 1
  done
done
cat "$out"
