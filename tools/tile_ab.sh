cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/tab
for L in A B; do
  if [ $L = B ]; then export SANTA_HIP_LIB=tools/ab/libsanta_hip_head.so; else unset SANTA_HIP_LIB; fi
  for r in 0 10; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/tab/$L$r -o t --output-format csv -- python3 -u tools/probe.py --phase solve --reps 5 --state-round $r > gpurun_out/tab/$L$r.json || exit 1
  done
done
echo ok
