#!/bin/bash
# round-5 GPU session: santa_lb_kernel with deferred candidate loads (LB_DEFER):
# large-block parity, then A/B against the synchronous staging (LB_DEFER=0)
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -q --timeout 600 --timeout-method thread \
  -k "reference_sizes or reference_block or wave_configs or round_vs_oracle or design or solve_round" \
  > gpurun_out/r5s_tests.log 2>&1 || { grep -E "Error|error|assert|FAIL" gpurun_out/r5s_tests.log | head -30; exit 1; }
tail -1 gpurun_out/r5s_tests.log
bash tools/ab_libs.sh gpurun_out/r5s_ab.jsonl \
  "--n 2000 --blocks 1 --phase solve --reps 3" "--n 2000 --phase solve --reps 2" "--n 2000 --phase solve --reps 2 --state-round 10" \
  -- abl/libsanta_hip_lbsync.so abl/libsanta_hip_lbdefer.so > gpurun_out/r5s_ab.log 2>&1 || { tail gpurun_out/r5s_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5s_ab.log | cut -c1-200
timeout -k 10 300 python -u tools/probe.py --n 2000 --blocks 1 --phase solve --reps 1 --lb-segments > gpurun_out/r5s_lb_segments_lone.json 2>/dev/null || exit 1
timeout -k 10 400 python -u bench.py --n 2000 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r5s_bench_n2000.json 2> gpurun_out/r5s_bench_n2000.err || { tail gpurun_out/r5s_bench_n2000.err; exit 1; }
cut -c1-260 gpurun_out/r5s_bench_n2000.json
echo all-done
