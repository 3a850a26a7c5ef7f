#!/bin/bash
cd $GRAFT_REPO_ROOT
for args in "--blocks 256" "--blocks 1024" "--blocks 2048" "" "--budget 23000" "--budget 27000" "--budget 32000" "--budget 40000" "--flags 32 --blocks 256" "--flags 32 --blocks 1024" "--flags 16 --blocks 256"; do
  echo "ARGS $args"
  timeout -k 10 120 python -u tools/probe.py --reps 2 $args 2>&1 | grep -v amdgpu.ids || exit 1
done
mkdir -p gpurun_out/pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/pmc -o sq1 --output-format csv -- python3 -u tools/probe.py --phase solve --reps 1 > gpurun_out/pmc/probe_sq1.json || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d gpurun_out/pmc -o sq2 --output-format csv -- python3 -u tools/probe.py --phase solve --reps 1 > gpurun_out/pmc/probe_sq2.json || exit 1
echo sweep done
