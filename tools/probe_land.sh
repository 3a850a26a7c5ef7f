mkdir -p gpurun_out
P="timeout -k 10 120 python -u tools/probe.py --phase solve --reps 3"
{ $P --mode 1 && $P --mode 1 --state-round 5 && $P --blocks 466 && $P --blocks 466 --state-round 10 && $P --blocks 933 && $P --blocks 933 --state-round 10 && $P --blocks 1865 && $P --blocks 1865 --state-round 10 && $P --blocks 3730 --state-round 10; } > gpurun_out/probe_land.log 2>&1
rc=$?; grep '^{' gpurun_out/probe_land.log; exit $rc
