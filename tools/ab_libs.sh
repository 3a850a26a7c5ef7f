#!/bin/bash
# A/B of kernel libraries on the same box: tools/ab_libs.sh OUT.jsonl "probe args"... -- lib1 lib2 ...
# (each probe runs once per library per repetition, alternating)
cd "$(dirname "$0")/.." || exit 2
out=$1; shift
probes=(); while [ "$1" != "--" ]; do probes+=("$1"); shift; done; shift
: > "$out"
for rep in 1 2; do
  for args in "${probes[@]}"; do
    for lib in "$@"; do
      r=$(SANTA_HIP_LIB=$lib timeout -k 10 120 python tools/probe.py $args) || exit 1
      echo "{\"lib\": \"$lib\", \"args\": \"$args\", \"r\": $r}" >> "$out"
      echo "$(basename $lib) [$args] $(echo $r | cut -c1-80)"
    done
  done
done
