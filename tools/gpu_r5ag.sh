#!/bin/bash
# round-5 GPU session: the 4-wave twins step-word ring offset in a VGPR, one word re-armed per step:
# parity, A/B against HEAD, twins bench both ways
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "twin or reference_sizes or reference_block or bench_rounds or round_vs_oracle or solve_round" > gpurun_out/r5ag_tests.log 2>&1 || { grep -E "Error|error|assert|FAIL" gpurun_out/r5ag_tests.log | head -30; exit 1; }
tail -1 gpurun_out/r5ag_tests.log
bash tools/ab_libs.sh gpurun_out/r5ag_ab.jsonl \
  "--mode 1 --phase solve --reps 5" "--mode 1 --phase solve --reps 5 --state-round 10" "--mode 1 --blocks 1 --phase solve --reps 5" \
  -- abl/libsanta_hip_a.so abl/libsanta_hip_b.so > gpurun_out/r5ag_ab.log 2>&1 || { tail gpurun_out/r5ag_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5ag_ab.log | cut -c1-150
for lib in a b a b; do
  SANTA_HIP_LIB=$PWD/abl/libsanta_hip_$lib.so timeout -k 10 300 python -u bench.py --mode twins --no-cpu-baseline >> gpurun_out/r5ag_bench_$lib.jsonl 2> gpurun_out/r5ag_bench.err || { tail gpurun_out/r5ag_bench.err; exit 1; }
done
for lib in a b; do python3 -c "
import json
for l in open('gpurun_out/r5ag_bench_$lib.jsonl'): d=json.loads(l); print('$lib', d['ms_per_step'], d['value'])
"; done
echo all-done
