#!/bin/bash
# rocprofv3 kernel trace + stats of the twins bench (run on the GPU box).
set -e
TAG=${1:-r01}
OUT=gpurun_out/prof_twins_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --mode twins > $OUT/bench_twins.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o trace --output-format csv -- \
    python3 -u bench.py --mode twins --no-cpu-baseline > $OUT/bench_under_trace.json
echo done
