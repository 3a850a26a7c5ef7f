#!/bin/bash
# Solve-kernel time of one rank's shard at N = 1, 2, 4, 8 (3730 / N blocks of
# the singles round), at round 0 and at the round-10 state (run on the GPU
# box).  One JSON line per case into $1 (default gpurun_out/shard_probe.jsonl).
OUT=${1:-gpurun_out/shard_probe.jsonl}
: > "$OUT"
for nb in 3730 1865 933 466; do
  for sr in 0 10; do
    args="--blocks $nb"
    [ $sr -ne 0 ] && args="$args --state-round $sr"
    line=$(timeout -k 10 120 python -u tools/probe.py --phase solve --reps 3 $args | tail -1) || exit $?
    python3 -c 'import json,sys; d=json.loads(sys.argv[2]); print(json.dumps({"args": sys.argv[1], "ms": round(min(d["solve"]["all_ms"]), 4), "steps_total": d["steps_total"]}))' "$args" "$line" >> "$OUT" || exit 1
  done
done
cat "$OUT"
