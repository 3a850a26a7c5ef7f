#!/bin/bash
# round-5 GPU session: santa_sp3_kernel one-word stores: lanes 1..63 to their own dump slot
# parity, A/B against HEAD (abl/libsanta_hip_a.so), bench
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "bench_rounds or round_vs_oracle or designs_agree or sparse_overflow or edge_block or argmin_agree or solve_round" \
  > gpurun_out/r5af_tests.log 2>&1 || { grep -E "Error|error|assert|FAIL" gpurun_out/r5af_tests.log | head -30; exit 1; }
tail -1 gpurun_out/r5af_tests.log
bash tools/ab_libs.sh gpurun_out/r5af_ab.jsonl \
  "--phase solve --reps 5" "--phase solve --reps 5 --state-round 10" "--blocks 1 --flags 128 --phase solve --reps 5" \
  -- abl/libsanta_hip_a.so abl/libsanta_hip_b.so > gpurun_out/r5af_ab.log 2>&1 || { tail gpurun_out/r5af_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5af_ab.log | cut -c1-160
for lib in a b a b; do
  SANTA_HIP_LIB=$PWD/abl/libsanta_hip_$lib.so timeout -k 10 300 python -u bench.py --no-cpu-baseline >> gpurun_out/r5af_bench_$lib.jsonl 2> gpurun_out/r5af_bench.err || { tail gpurun_out/r5af_bench.err; exit 1; }
done
for lib in a b; do python3 -c "
import json,sys
for l in open('gpurun_out/r5af_bench_$lib.jsonl'): d=json.loads(l); print('$lib', d['ms_per_step'], d['value'])
"; done
bash tools/pmc_probe.sh > gpurun_out/r5af_pmc.log 2>&1 || { tail gpurun_out/r5af_pmc.log; exit 1; }
echo all-done
