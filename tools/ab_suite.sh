#!/bin/bash
# A/B latency suite of two library builds on one box (dev tool):
#   tools/ab_suite.sh <lib_b.so> [reps]
# A = the in-tree libsanta_hip.so, B = the given build.  Workloads: the
# singles full round (3730 blocks, sparse kernel) at rounds 0 and 10, one
# GPU's 8-GPU shard (466 blocks, 4-wave LDS tile) at rounds 0 and 10, the
# twins round (78 blocks) at round 0, and lone blocks (sparse / LDS tile).
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
B=$1; R=${2:-2}
run() {  # label lib args...
  local lab=$1 lib=$2; shift 2
  SANTA_HIP_LIB=${lib:-$SANTA_HIP_LIB} timeout -k 10 120 python -u tools/probe.py --phase solve --reps 3 "$@" > gpurun_out/ab1.json || exit $?
  python3 -c "
import json; d = json.load(open('gpurun_out/ab1.json'))
print(json.dumps({'lib': '$lab', 'args': '$*', 'ms': round(d['solve']['ms'], 4), 'steps_max': d['steps_max'],
                  'steps_total': d['steps_total']}))"
}
for rep in $(seq 1 "$R"); do
  for w in "--blocks 3730" "--blocks 3730 --state-round 10" "--blocks 466" "--blocks 466 --state-round 10" \
           "--mode 1" "--blocks 1 --flags 128" "--blocks 1 --flags 8"; do
    run A "" $w
    run B "$B" $w
  done
done
