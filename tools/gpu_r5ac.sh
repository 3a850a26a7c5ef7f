#!/bin/bash
# round-5 GPU session: sap_solve_mw (large blocks, triplets, batched LSAP) with
# the next row from the step word's VGPR copy: parity, A/B against HEAD
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -q --timeout 600 --timeout-method thread \
  -k "reference_sizes or reference_block or wave_configs or triplet or lsap or big or round_vs_oracle" \
  > gpurun_out/r5ac_tests.log 2>&1 || { grep -E "Error|error|assert|FAIL" gpurun_out/r5ac_tests.log | head -30; exit 1; }
tail -1 gpurun_out/r5ac_tests.log
for lib in a b a b; do
  echo "== $lib" >> gpurun_out/r5ac_lsap.log
  SANTA_HIP_LIB=$PWD/abl/libsanta_hip_$lib.so timeout -k 10 300 python -u tools/lsap_time.py 256x4096 512x256 1024x256 >> gpurun_out/r5ac_lsap.log 2>/dev/null || exit 1
done
grep -v amdgpu gpurun_out/r5ac_lsap.log
for lib in a b; do
  SANTA_HIP_LIB=$PWD/abl/libsanta_hip_$lib.so timeout -k 10 400 python -u bench.py --mode twins --n 3000 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r5ac_bench_tw3000_$lib.json 2> gpurun_out/r5ac_bench.err || { tail gpurun_out/r5ac_bench.err; exit 1; }
  SANTA_HIP_LIB=$PWD/abl/libsanta_hip_$lib.so timeout -k 10 300 python -u bench.py --mode triplets --no-cpu-baseline > gpurun_out/r5ac_bench_tri_$lib.json 2>> gpurun_out/r5ac_bench.err || { tail gpurun_out/r5ac_bench.err; exit 1; }
  python3 -c "
import json
for f in ('tw3000','tri'):
    d=json.loads(open('gpurun_out/r5ac_bench_'+f+'_$lib.json').read().strip().splitlines()[-1]); print('$lib', f, d['ms_per_step'], d['roofline']['latency']['cycles_per_step_lone'])"
done
echo all-done
