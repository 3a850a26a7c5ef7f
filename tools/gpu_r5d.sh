#!/bin/bash
# round-5 GPU session: santa_lb_kernel parity subset, then its segment profile
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "reference_sizes or round_vs_oracle or wave_configs or design_dispatch" \
  > gpurun_out/r5d_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" gpurun_out/r5d_tests.log | tail -40; exit 1; }
tail -2 gpurun_out/r5d_tests.log
bash tools/gpu_r5c.sh
