#!/bin/bash
# round-4 GPU session 23: side-stream sampling that may only start on a CU
# once the solve has freed LDS there (the sampler launch reserves 8 / 16 KB
# of LDS: abl/sl*.hip), against in-line sampling (tools/gap_probe.py loops)
cd /root/repo
for lib in sl0 sl8 sl16; do
  SANTA_HIP_LIB=abl/$lib.so timeout -k 10 300 python tools/gap_probe.py --rounds 60 --reps 4 \
    --only loop_p0_side,loop_p1_side,loop_p2_side > gpurun_out/gap_r4w_$lib.json || exit 1
  echo $lib; cat gpurun_out/gap_r4w_$lib.json | cut -c1-260
done
echo all-done
