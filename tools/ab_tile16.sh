#!/bin/bash
# A/B: tile build with 16-byte wishlist window loads (libsanta_hip.so) vs head
cd "$(dirname "$0")/.." || exit 2
H=mpi-hungarian-method_amd/santa_hip/libsanta_head.so; N=mpi-hungarian-method_amd/santa_hip/libsanta_hip.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t16_tests.log 2>&1 || { tail -30 gpurun_out/t16_tests.log; exit 1; }
tail -2 gpurun_out/t16_tests.log
bash tools/ab_libs.sh gpurun_out/ab_tile16.jsonl "--phase solve --reps 5" "--phase solve --reps 5 --state-round 10" -- $H $N || exit 1
for L in $H $N; do SANTA_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/t16_$(basename $L .so) -o tr --output-format csv -- python3 -u tools/probe.py --phase solve --reps 3 > /dev/null || exit 1; done
echo done
