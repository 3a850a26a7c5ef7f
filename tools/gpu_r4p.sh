#!/bin/bash
# round-4 GPU session 16: the driver with in-line sampling and the side-stream
# bookkeeping: driver parity, then an alternating bench A/B against the r04b
# driver (abl/driver_r04b.py), 20-step (the driver's default) and 100-step runs
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "pipelined or bench_rounds or ranks or trajectory or exchange_over_rccl or cli_rounds" \
  > gpurun_out/tests_r4p.log 2>&1 || { tail -30 gpurun_out/tests_r4p.log; exit 1; }
tail -2 gpurun_out/tests_r4p.log
old=/tmp/old_tree
mkdir -p $old && tar --exclude=./gpurun_out --exclude=./abl -cf - . | tar -C $old -xf - || exit 1
cp abl/driver_r04b.py $old/mpi-hungarian-method_amd/santa_hip/driver.py || exit 1
: > gpurun_out/ab_r4p.jsonl
for rep in 1 2 3; do
  for side in new old; do
    dir=/root/repo; [ $side = old ] && dir=$old
    for cfg in "single 20" "single 100" "twins 20"; do
      set -- $cfg
      r=$(cd $dir && timeout -k 10 180 python bench.py --no-cpu-baseline --steps $2 --warmup 3 --mode $1) || exit 1
      echo "{\"side\": \"$side\", \"mode\": \"$1\", \"steps\": $2, \"r\": $r}" >> gpurun_out/ab_r4p.jsonl
      echo "$side $1 $2 $(echo $r | grep -o '"ms_per_step": [0-9.]*')"
    done
  done
done
echo all-done
