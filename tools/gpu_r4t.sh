#!/bin/bash
# round-4 GPU session 20: the N > 1 round loop over a real RCCL group (one
# rank), then the bench lines of the final driver (singles and twins with the
# CPU baselines) on the profiled kernel source
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "exchange_over_rccl or two_ranks or pipelined" > gpurun_out/tests_r4t.log 2>&1 || { tail -30 gpurun_out/tests_r4t.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/tests_r4t.log | cut -c1-120
timeout -k 10 400 python bench.py > gpurun_out/bench_r4t_single.json 2> gpurun_out/bench_r4t_single.err || exit 1
timeout -k 10 400 python bench.py --mode twins > gpurun_out/bench_r4t_twins.json 2> gpurun_out/bench_r4t_twins.err || exit 1
cut -c1-400 gpurun_out/bench_r4t_single.json gpurun_out/bench_r4t_twins.json
echo all-done
