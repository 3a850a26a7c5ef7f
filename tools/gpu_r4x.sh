#!/bin/bash
# round-4 GPU session 24: kernel trace of the bench with the final round loop
# (the between-rounds gap; the kernel source is the profiled c54608004b3b2d8c)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/prof_r04g -o trace --output-format csv -- \
  python3 /root/repo/bench.py --no-cpu-baseline --steps 20 --warmup 3 > /root/repo/gpurun_out/prof_r04g.log 2>&1 || exit 1
echo all-done
