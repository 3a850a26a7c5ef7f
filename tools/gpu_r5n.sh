#!/bin/bash
# round-5 GPU session: publish fast path (empty fallback list) + sampled bench events
# (the loop with / without the mailbox and the fused sampling), the bench and
# a kernel trace for the between-round gap
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "mailbox or solve_round or bench_rounds_vs_oracle or trajectory or pipelined or rccl or two_ranks" \
  > gpurun_out/r5n_tests.log 2>&1 || { grep -E "Error|error|assert|FAIL" gpurun_out/r5n_tests.log | head -30; exit 1; }
tail -1 gpurun_out/r5n_tests.log
timeout -k 10 400 python tools/gap_probe.py --rounds 40 --reps 3 --only bare,loop_r5,loop_r5_nomail \
  > gpurun_out/r5n_gap_probe.json 2> gpurun_out/r5n_gap_probe.err || { tail gpurun_out/r5n_gap_probe.err; exit 1; }
cut -c1-400 gpurun_out/r5n_gap_probe.json
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r5n_bench.json 2> gpurun_out/r5n_bench.err || { tail gpurun_out/r5n_bench.err; exit 1; }
cut -c1-300 gpurun_out/r5n_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5n_trace -o bench -- python bench.py --no-cpu-baseline > gpurun_out/r5n_trace.log 2>&1 || { tail gpurun_out/r5n_trace.log; exit 1; }
python tools/round_gaps.py $(find gpurun_out/r5n_trace -name "*kernel_trace.csv" | head -1) santa_sp3_kernel r05n
echo all-done
