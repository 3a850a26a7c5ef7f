#!/bin/bash
# round-5 GPU session 2: santa_lb_kernel (staged candidate rows, lattice
# units) -- the large-block parity tests first, then lone / full-round probes
# against the row-rebuild kernel (SH_FLAG_BIG_ROWS = 8192)
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread \
  -k "reference_sizes or round_vs_oracle or wave_configs or design_dispatch" \
  > gpurun_out/r5b_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" gpurun_out/r5b_tests.log | tail -40; exit 1; }
grep -cE "PASSED" gpurun_out/r5b_tests.log; tail -2 gpurun_out/r5b_tests.log
for fl in 0 8192; do
  timeout -k 10 120 python tools/probe.py --n 2000 --blocks 1 --phase solve --reps 3 --flags $fl | cut -c1-200 || exit 1
done
for fl in 0 8192; do
  timeout -k 10 200 python tools/probe.py --n 2000 --phase solve --reps 2 --flags $fl | cut -c1-200 || exit 1
done
timeout -k 10 200 python tools/probe.py --n 2000 --phase solve --reps 2 --state-round 10 | cut -c1-200 || exit 1
echo all-done
