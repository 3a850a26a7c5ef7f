#!/bin/bash
# GPU-box session: twins bench with its CPU baseline, and a 2-rank bench
# rehearsal on one GPU (gloo) of the distributed exchange path.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --mode twins > gpurun_out/bench_twins_cpu.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_twins_cpu.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29555 bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo --one-device \
  > gpurun_out/bench_2rank_gloo.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_2rank_gloo.log
