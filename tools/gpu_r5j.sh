#!/bin/bash
# round-5 GPU session: sh_solve_round (fused undo + next-round sampling):
# the new test and the whole suite, bench lines and a kernel trace for the gap
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "solve_round_bookkeeping" \
  > gpurun_out/r5j_new.log 2>&1 || { grep -E "Error|error|assert|FAIL" gpurun_out/r5j_new.log | head -30; exit 1; }
tail -1 gpurun_out/r5j_new.log
bash tools/gpu_run.sh tests > gpurun_out/r5j_tests_step.log 2>&1 || { tail -40 gpurun_out/r5j_tests_step.log; exit 1; }
grep -E "passed|failed" gpurun_out/tests.log | tail -2
grep -q " failed" gpurun_out/tests.log && exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r5j_bench.json 2> gpurun_out/r5j_bench.err || { tail gpurun_out/r5j_bench.err; exit 1; }
cut -c1-300 gpurun_out/r5j_bench.json
timeout -k 10 300 python -u bench.py --mode twins --no-cpu-baseline > gpurun_out/r5j_bench_twins.json 2> gpurun_out/r5j_bench_twins.err || { tail gpurun_out/r5j_bench_twins.err; exit 1; }
cut -c1-300 gpurun_out/r5j_bench_twins.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5j_trace -o bench -- python bench.py --no-cpu-baseline > gpurun_out/r5j_trace.log 2>&1 || { tail gpurun_out/r5j_trace.log; exit 1; }
python tools/round_gaps.py $(find gpurun_out/r5j_trace -name "*kernel_trace.csv" | head -1) santa_sp3_kernel r05j
echo all-done
