#!/bin/bash
# A/B latency probe of two library builds on the same box (dev tool):
#   tools/ab_probe.sh <lib_b.so> <probe args...>
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
B=$1; shift
for rep in 1 2; do
  for lib in "" "$B"; do
    SANTA_HIP_LIB=$lib timeout -k 10 120 python -u tools/probe.py --phase solve --reps 5 "$@" > gpurun_out/ab.json || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));print('${lib:-A}', d['blocks'], d['state_round'], round(d.get('solve', d.get('score'))['ms'],4))"
  done
done
