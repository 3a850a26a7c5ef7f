#!/bin/bash
# round-5 GPU session: twins at n = 256 -- the 4-wave step's segments
# (SH_FLAG_TIMING on sap_solve_mw_sc, the TWINS_1W=0 build) and the one-wave
# solve (TWINS_1W=1): parity, A/B of the round and the lone block, bench lines
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "twin or bench_rounds or round_vs_oracle or designs or solve_round" > gpurun_out/r5r_tests.log 2>&1 || { grep -E "Error|error|assert|FAIL" gpurun_out/r5r_tests.log | head -30; exit 1; }
tail -1 gpurun_out/r5r_tests.log
rm -f gpurun_out/r5r_segments.jsonl
for A in "--mode 1 --blocks 1 --phase solve --reps 1 --segments" "--mode 1 --phase solve --reps 1 --segments" \
         "--mode 1 --phase solve --reps 1 --segments --state-round 10"; do
  SANTA_HIP_LIB=$PWD/abl/libsanta_hip_tw4.so timeout -k 10 300 python -u tools/probe.py $A >> gpurun_out/r5r_segments.jsonl 2>gpurun_out/r5r.err || { tail gpurun_out/r5r.err; exit 1; }
done
cut -c1-700 gpurun_out/r5r_segments.jsonl
bash tools/ab_libs.sh gpurun_out/r5r_ab.jsonl \
  "--mode 1 --phase solve --reps 5" "--mode 1 --phase solve --reps 5 --state-round 10" "--mode 1 --blocks 1 --phase solve --reps 5" \
  -- abl/libsanta_hip_tw4.so abl/libsanta_hip_tw1.so > gpurun_out/r5r_ab.log 2>&1 || { tail gpurun_out/r5r_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5r_ab.log
for lib in tw4 tw1; do
  SANTA_HIP_LIB=$PWD/abl/libsanta_hip_$lib.so timeout -k 10 300 python -u bench.py --mode twins --no-cpu-baseline > gpurun_out/r5r_bench_$lib.json 2> gpurun_out/r5r_bench_$lib.err || { tail gpurun_out/r5r_bench_$lib.err; exit 1; }
  cut -c1-260 gpurun_out/r5r_bench_$lib.json
done
echo all-done
