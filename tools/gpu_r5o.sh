#!/bin/bash
# round-5 GPU session: santa_big_kernel with each wave's candidate row loaded
# before the fold (BIG_STAGED) -- the large-block parity tests, then the
# 3000-pair twins and triplets bench A/B against the unstaged build
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -q --timeout 600 --timeout-method thread \
  -k "reference_sizes or reference_block or round_vs_oracle or wave_configs or big or large or triplet or solve_round or design" \
  > gpurun_out/r5o_tests.log 2>&1 || { grep -E "Error|error|assert|FAIL" gpurun_out/r5o_tests.log | head -30; exit 1; }
tail -1 gpurun_out/r5o_tests.log
for lib in staged nostaged; do
  if [ $lib = nostaged ]; then export SANTA_HIP_LIB=$PWD/abl/libsanta_hip_nostaged.so; fi
  timeout -k 10 300 python -u bench.py --mode twins --n 3000 --steps 5 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r5o_twins3000_$lib.json 2> gpurun_out/r5o_twins3000_$lib.err || { tail gpurun_out/r5o_twins3000_$lib.err; exit 1; }
  cut -c1-200 gpurun_out/r5o_twins3000_$lib.json
done
unset SANTA_HIP_LIB
echo all-done
