#!/bin/bash
# A/B: tile build from the 10-bit packed wishlist (libsanta_hip.so) vs the 16-byte window loads (head)
cd "$(dirname "$0")/.." || exit 2
H=mpi-hungarian-method_amd/santa_hip/libsanta_head.so; N=mpi-hungarian-method_amd/santa_hip/libsanta_hip.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/p10_tests.log 2>&1 || { tail -30 gpurun_out/p10_tests.log; exit 1; }
tail -2 gpurun_out/p10_tests.log
bash tools/ab_libs.sh gpurun_out/ab_pack10.jsonl "--phase solve --reps 5" "--phase solve --reps 5 --state-round 10" -- $H $N || exit 1
for L in $H $N; do SANTA_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p10_$(basename $L .so) -o tr --output-format csv -- python3 -u tools/probe.py --phase solve --reps 3 > /dev/null || exit 1; done
echo done
