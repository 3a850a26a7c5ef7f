#!/bin/bash
# round-4 GPU session 22: the next round's sampling overlapped with the
# all-gather (exchange's `during`): the N > 1 loop over RCCL (one rank),
# two ranks on the HIP path (gloo), the pipelined loop; a bench sanity run
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "exchange_over_rccl or two_ranks or pipelined or bench_rounds" > gpurun_out/tests_r4v.log 2>&1 || { tail -30 gpurun_out/tests_r4v.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/tests_r4v.log | cut -c1-100
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r4v.json 2> gpurun_out/bench_r4v.err || exit 1
cut -c1-200 gpurun_out/bench_r4v.json
echo all-done
