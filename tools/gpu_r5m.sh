#!/bin/bash
# round-5 GPU session: kernel traces of the gap probe's bare and loop variants
# (where the hole after the fallback launch comes from)
cd /root/repo
export TMPDIR=/tmp
for v in bare loop_r5 loop_r5_nomail; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5m_$v -o t -- python tools/gap_probe.py --rounds 30 --reps 1 --only $v \
    > gpurun_out/r5m_$v.log 2>&1 || { tail gpurun_out/r5m_$v.log; exit 1; }
done
echo all-done
