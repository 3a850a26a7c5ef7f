#!/bin/bash
# round-4 GPU session 21: issue priority back to 3 for a block whose steps
# since its last 32 Dijkstras began pass T (600 / 900 / 1300), against the
# position-only schedule (abl/pr*.hip, santa_sp3_kernel); full rounds 0, 10
cd /root/repo
bash tools/ab_libs.sh gpurun_out/ab_r4u.jsonl "--phase solve --reps 3" "--phase solve --reps 3 --state-round 10" \
  -- abl/pr_base.so abl/pr600.so abl/pr900.so abl/pr1300.so > gpurun_out/ab_r4u.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab_r4u.log | cut -c1-100
echo all-done
