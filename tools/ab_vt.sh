#!/bin/bash
cd /root/repo || exit 2
H=mpi-hungarian-method_amd/santa_hip/libsanta_head.so; N=mpi-hungarian-method_amd/santa_hip/libsanta_hip.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/vt_tests.log 2>&1 || { tail -30 gpurun_out/vt_tests.log; exit 1; }
tail -2 gpurun_out/vt_tests.log
bash tools/ab_libs.sh gpurun_out/ab_vt.jsonl "--phase solve --reps 5 --blocks 933" "--phase solve --reps 5 --blocks 933 --state-round 10" -- $H $N
