#!/bin/bash
# Dev A/B of library builds on the singles full round only (3730 blocks at
# state rounds 0 and 10): tools/ab_round.sh <reps> <lib_b.so>...
# A = the in-tree libsanta_hip.so; the builds are interleaved per repetition.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
R=$1; shift
for rep in $(seq 1 "$R"); do
  for w in "--blocks 3730" "--blocks 3730 --state-round 10"; do
    for lib in "" "$@"; do
      SANTA_HIP_LIB=${lib:-$SANTA_HIP_LIB} timeout -k 10 120 python -u tools/probe.py --phase solve --reps 3 $w > gpurun_out/ab1.json || exit $?
      python3 -c "
import json; d = json.load(open('gpurun_out/ab1.json'))
print(json.dumps({'lib': '$(basename "${lib:-A}")', 'args': '$w', 'ms': round(d['solve']['ms'], 4), 'steps_total': d['steps_total']}))"
    done
  done
done
