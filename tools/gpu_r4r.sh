#!/bin/bash
# round-4 GPU session 18: where the twins kernel's tile build time goes
# (ablation libraries from abl/tw_*.hip: no code->entry pass, no row stores,
# no gift-side epilogue reads; SH_FLAG_BUILD_ONLY launches, 78 blocks)
cd /root/repo
bash tools/ab_libs.sh gpurun_out/ab_r4r_twbuild.jsonl "--mode 1 --phase build --reps 5" \
  -- abl/tw_base.so abl/tw_norc2.so abl/tw_nostore.so abl/tw_noepi.so > gpurun_out/ab_r4r.log 2>&1 || exit 1
cat gpurun_out/ab_r4r.log
echo all-done
