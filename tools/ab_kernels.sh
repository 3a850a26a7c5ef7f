#!/bin/bash
# Per-kernel A/B (dev tool): rocprofv3 kernel stats of the full-round probe
# (rounds 0 and 10) for the in-tree library (A) and a given build (B).
#   tools/ab_kernels.sh <lib_b.so> [kernel-name regex]
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
B=$1; RX=${2:-"tile|sp2"}
for lab in A B; do
  lib=""; [ "$lab" = B ] && lib=$B
  for st in 0 10; do
    d=gpurun_out/abk_${lab}_$st
    SANTA_HIP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o p --output-format csv -- \
      python3 -u tools/probe.py --phase solve --reps 5 --state-round $st > /dev/null 2>&1 || exit 1
    python3 - "$lab" "$st" "$d/p_kernel_stats.csv" "$RX" <<'PY'
import csv, re, sys
lab, st, f, rx = sys.argv[1:]
for r in csv.DictReader(open(f)):
    if re.search(rx, r["Name"]):
        print(f"{lab} round {st}: {r['Name'][:60]} calls {r['Calls']} avg_us {float(r['AverageNs'])/1e3:.1f}")
PY
  done
done
