#!/bin/bash
# round-5 GPU session: the whole GPU suite on the round's source (lb kernel,
# undo protocol), a short bench per mode, and a kernel trace of the singles
# bench for the between-round gap
cd /root/repo
export TMPDIR=/tmp
bash tools/gpu_run.sh tests > gpurun_out/r5i_tests_step.log 2>&1 || { tail -40 gpurun_out/r5i_tests_step.log; exit 1; }
grep -E "passed|failed" gpurun_out/tests.log | tail -2
grep -q " failed" gpurun_out/tests.log && exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r5i_bench.json 2> gpurun_out/r5i_bench.err || { tail gpurun_out/r5i_bench.err; exit 1; }
cut -c1-400 gpurun_out/r5i_bench.json
timeout -k 10 300 python -u bench.py --mode twins --no-cpu-baseline > gpurun_out/r5i_bench_twins.json 2> gpurun_out/r5i_bench_twins.err || { tail gpurun_out/r5i_bench_twins.err; exit 1; }
cut -c1-300 gpurun_out/r5i_bench_twins.json
timeout -k 10 300 python -u bench.py --n 2000 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r5i_bench_n2000.json 2> gpurun_out/r5i_bench_n2000.err || { tail gpurun_out/r5i_bench_n2000.err; exit 1; }
cut -c1-300 gpurun_out/r5i_bench_n2000.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5i_trace -o bench -- python bench.py --no-cpu-baseline > gpurun_out/r5i_trace.log 2>&1 || { tail gpurun_out/r5i_trace.log; exit 1; }
python tools/round_gaps.py $(find gpurun_out/r5i_trace -name "*kernel_trace.csv" | head -1) santa_sp3_kernel r05i
echo all-done
