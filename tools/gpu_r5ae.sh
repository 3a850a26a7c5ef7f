#!/bin/bash
# round-5 GPU session: santa_lb_kernel minVal from the word VGPR copy:
# (the candidate's slot selected per lane in VALU, wave-uniform stores):
# large-block parity, A/B against HEAD, n = 2000 bench both ways
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -q --timeout 600 --timeout-method thread \
  -k "reference_sizes or reference_block or wave_configs or round_vs_oracle or design or solve_round" \
  > gpurun_out/r5ae_tests.log 2>&1 || { grep -E "Error|error|assert|FAIL" gpurun_out/r5ae_tests.log | head -30; exit 1; }
tail -1 gpurun_out/r5ae_tests.log
bash tools/ab_libs.sh gpurun_out/r5ae_ab.jsonl \
  "--n 2000 --blocks 1 --phase solve --reps 3" "--n 2000 --phase solve --reps 2" "--n 2000 --phase solve --reps 2 --state-round 10" \
  -- abl/libsanta_hip_a.so abl/libsanta_hip_b.so > gpurun_out/r5ae_ab.log 2>&1 || { tail gpurun_out/r5ae_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5ae_ab.log | cut -c1-160
for lib in a b; do
  SANTA_HIP_LIB=$PWD/abl/libsanta_hip_$lib.so timeout -k 10 400 python -u bench.py --n 2000 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r5ae_bench_$lib.json 2> gpurun_out/r5ae_bench.err || { tail gpurun_out/r5ae_bench.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r5ae_bench_$lib.json').read().strip().splitlines()[-1]); print('$lib', d['ms_per_step'], d['roofline']['latency']['cycles_per_step_lone'])"
done
echo all-done
