#!/bin/bash
# round-5 GPU session: santa_sp3_kernel with conflict-free ds_read_b64 row reads
# (and a cheaper augmentation guard): parity, then A/B against the r5n build
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "bench_rounds or round_vs_oracle or designs_agree or sparse_overflow or edge_block or argmin_agree or solve_round" \
  > gpurun_out/r5q_tests.log 2>&1 || { grep -E "Error|error|assert|FAIL" gpurun_out/r5q_tests.log | head -30; exit 1; }
tail -1 gpurun_out/r5q_tests.log
bash tools/ab_libs.sh gpurun_out/r5q_ab.jsonl \
  "--phase solve --reps 5" "--phase solve --reps 5 --state-round 10" "--blocks 1 --flags 128 --phase solve --reps 5" \
  -- abl/libsanta_hip_r5n.so abl/libsanta_hip_r5q.so > gpurun_out/r5q_ab.log 2>&1 || { tail gpurun_out/r5q_ab.log; exit 1; }
cat gpurun_out/r5q_ab.log
for lib in r5n r5q; do
  SANTA_HIP_LIB=$PWD/abl/libsanta_hip_$lib.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r5q_bench_$lib.json 2> gpurun_out/r5q_bench_$lib.err || { tail gpurun_out/r5q_bench_$lib.err; exit 1; }
  cut -c1-260 gpurun_out/r5q_bench_$lib.json
done
echo all-done
