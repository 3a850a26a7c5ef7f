#!/bin/bash
# Round-end evidence on the current source (GPU box): tests, smoke, rocprofv3 profiles
# (tag r02g), bench lines for every mode, n=2000 convergence through the CLI.
cd "$(dirname "$0")/.." || exit 2
bash tools/gpu_run.sh tests smoke > gpurun_out/final_ts.log 2>&1 || exit 1
grep -q " passed" gpurun_out/tests.log && ! grep -q " failed" gpurun_out/tests.log || exit 1
bash tools/profile_round.sh r02g single > gpurun_out/prof_r02g.log 2>&1 || exit 1
bash tools/profile_round.sh r02gt twins > gpurun_out/prof_r02gt.log 2>&1 || exit 1
bash tools/gpu_run.sh bench bench_twins bench_triplets bench_n2000 > gpurun_out/final_bench.log 2>&1 || exit 1
cd mpi-hungarian-method_amd && timeout -k 10 300 python -u -m santa_hip.driver --block-size 2000 --rounds 40 --patience 3 > ../gpurun_out/conv_single_n2000.jsonl 2>/dev/null
echo final-done
