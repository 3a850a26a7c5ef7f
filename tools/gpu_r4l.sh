#!/bin/bash
# round-4 GPU session 12: the round's bookkeeping moved off the round's
# stream (driver.py: sampling two rounds ahead, the delta's host copy on the
# side stream, no waits on completed events).  Pipelined/delta parity, then an
# alternating bench A/B against the r04b driver (abl/driver_r04b.py), then a
# kernel trace of the new round loop.
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "pipelined or bench_rounds or delta or reference_block_sizes or twins_rounds or dist" \
  > gpurun_out/tests_r4l.log 2>&1 || { tail -30 gpurun_out/tests_r4l.log; exit 1; }
tail -2 gpurun_out/tests_r4l.log
old=/tmp/old_tree
mkdir -p $old && tar --exclude=./gpurun_out --exclude=./abl -cf - . | tar -C $old -xf - || exit 1
cp abl/driver_r04b.py $old/mpi-hungarian-method_amd/santa_hip/driver.py || exit 1
: > gpurun_out/ab_r4l.jsonl
for rep in 1 2 3; do
  for side in new old; do
    dir=/root/repo; [ $side = old ] && dir=$old
    for mode in single twins; do
      r=$(cd $dir && timeout -k 10 180 python bench.py --no-cpu-baseline --steps 100 --warmup 5 --mode $mode) || exit 1
      echo "{\"side\": \"$side\", \"mode\": \"$mode\", \"r\": $r}" >> gpurun_out/ab_r4l.jsonl
      echo "$side $mode $(echo $r | grep -o '"ms_per_step": [0-9.]*')"
    done
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/prof_r04l -o trace -- \
  python3 /root/repo/bench.py --no-cpu-baseline --steps 20 --warmup 3 > /root/repo/gpurun_out/prof_r04l.log 2>&1 || exit 1
echo all-done
