#!/bin/bash
# dev: SQ counters of the block kernel for one probe configuration (two passes)
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pmc; mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $OUT -o sq1 --output-format csv -- python3 -u tools/probe.py --phase solve --reps 1 "$@" > $OUT/probe_sq1.json || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU -d $OUT -o sq2 --output-format csv -- python3 -u tools/probe.py --phase solve --reps 1 "$@" > $OUT/probe_sq2.json || exit 1
echo pmc done
