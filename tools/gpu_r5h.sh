#!/bin/bash
# round-5 GPU session: the masked dual update of the one-wave kernels
# (VERDICT r04 next #2): dv1 = round 4's variant (kernel trace: where the
# time goes), dv2 = dense-tile kernel with the sink included, sv2 = the same
# in santa_sp3_kernel; parity, then A/B against dv0 (= the default library)
cd /root/repo
export TMPDIR=/tmp
for v in dv2 sv2; do
  SANTA_HIP_LIB=abl/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread \
    -k "round_vs_oracle or shard_designs or kernel_designs or bench_rounds_vs_oracle" > gpurun_out/r5h_tests_$v.log 2>&1 || { echo "FAIL $v"; tail -30 gpurun_out/r5h_tests_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r5h_tests_$v.log)"
done
SANTA_HIP_LIB=abl/dv1.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r5h_dv1 -o dv1 -- python tools/probe.py --blocks 466 --phase solve --reps 2 --state-round 10 > gpurun_out/r5h_dv1_probe.log 2>&1 || { tail -20 gpurun_out/r5h_dv1_probe.log; exit 1; }
find gpurun_out/r5h_dv1 -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-8 {} | head -8'
bash tools/ab_libs.sh gpurun_out/r5h_ab.jsonl "--blocks 466 --phase solve --reps 3" "--blocks 466 --phase solve --reps 3 --state-round 10" \
  "--blocks 1 --flags 4096 --phase solve --reps 3" -- abl/dv0.so abl/dv2.so > gpurun_out/r5h_ab.log 2>&1 || { tail -20 gpurun_out/r5h_ab.log; exit 1; }
bash tools/ab_libs.sh gpurun_out/r5h_ab_sp3.jsonl "--phase solve --reps 3" "--phase solve --reps 3 --state-round 10" \
  "--blocks 1 --flags 128 --phase solve --reps 3" -- abl/dv0.so abl/sv2.so > gpurun_out/r5h_ab_sp3.log 2>&1 || { tail -20 gpurun_out/r5h_ab_sp3.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5h_ab.log gpurun_out/r5h_ab_sp3.log | cut -c1-140
echo all-done
