#!/bin/bash
# round-4 GPU session 17: bench A/B of the driver's sampling placement
# (PREFETCH 0 = in line, 2 = two rounds ahead on the side stream) against the
# r04b driver, alternating, 100-step and 20-step singles runs
cd /root/repo
for v in p2 old; do
  t=/tmp/tree_$v
  mkdir -p $t && tar --exclude=./gpurun_out --exclude=./abl -cf - . | tar -C $t -xf - || exit 1
done
sed -i 's/^    PREFETCH = 0$/    PREFETCH = 2/' /tmp/tree_p2/mpi-hungarian-method_amd/santa_hip/driver.py
grep -c "^    PREFETCH = 2$" /tmp/tree_p2/mpi-hungarian-method_amd/santa_hip/driver.py || exit 1
cp abl/driver_r04b.py /tmp/tree_old/mpi-hungarian-method_amd/santa_hip/driver.py || exit 1
: > gpurun_out/ab_r4q.jsonl
for rep in 1 2 3 4; do
  for side in p0 p2 old; do
    dir=/root/repo; [ $side != p0 ] && dir=/tmp/tree_$side
    for st in 100 20; do
      r=$(cd $dir && timeout -k 10 180 python bench.py --no-cpu-baseline --steps $st --warmup 3) || exit 1
      echo "{\"side\": \"$side\", \"steps\": $st, \"r\": $r}" >> gpurun_out/ab_r4q.jsonl
      echo "$side $st $(echo $r | grep -o '"ms_per_step": [0-9.]*')"
    done
  done
done
echo all-done
