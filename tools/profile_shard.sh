#!/bin/bash
# rocprofv3 evidence for one GPU's shard at N = 8 (466 blocks, the 4-wave LDS-tile
# kernel, round-0 state): kernel trace + the SQ / occupancy PMC passes of
# tools/profile_round.sh, each pass its own run.  Then locally:
#   python tools/summarize_profile.py gpurun_out/prof_<tag> <tag>
set -e
TAG=${1:-r03s}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P="python3 -u tools/probe.py --phase solve --reps 1 --blocks 466"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o trace --output-format csv -- $P > $OUT/probe_trace.json
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $OUT -o sq1 --output-format csv -- \
    $P > $OUT/probe_sq1.json
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $OUT -o sq2 --output-format csv -- \
    $P > $OUT/probe_sq2.json
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $OUT -o occ --output-format csv -- \
    $P > $OUT/probe_occ.json
echo done
