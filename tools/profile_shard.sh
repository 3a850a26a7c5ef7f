#!/bin/bash
# rocprofv3 evidence for rank 0's shard of a multi-GPU singles round (round-0
# state): kernel trace + the HBM (FETCH_SIZE / WRITE_SIZE), SQ and occupancy
# PMC passes of tools/profile_round.sh, each pass its own run.
#   tools/profile_shard.sh r03s8 467    # N = 8: 4-wave LDS-tile kernel
#   tools/profile_shard.sh r03s4 933    # N = 4: 4-wave register-tile kernel
#   tools/profile_shard.sh r03s2 1865   # N = 2: register-tile sparse design
# (rank 0 holds ceil(3730 / N) blocks, driver.shard_range).  Then locally:
#   python tools/summarize_profile.py gpurun_out/prof_<tag> <tag>
# bench.py takes a summary's traffic / occupancy only for a launch of the
# same size (summary probe.blocks == the rank's blocks).
set -e
TAG=${1:-r03s8}
BLOCKS=${2:-467}
EXTRA=${3:-}   # more probe arguments, e.g. "--n 2000" (the reference's block size)
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P="python3 -u tools/probe.py --phase solve --reps 1 --blocks $BLOCKS $EXTRA"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o trace --output-format csv -- $P > $OUT/probe_trace.json
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT -o fetch --output-format csv -- $P > $OUT/probe_fetch.json
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT -o write --output-format csv -- $P > $OUT/probe_write.json
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $OUT -o sq1 --output-format csv -- \
    $P > $OUT/probe_sq1.json
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $OUT -o sq2 --output-format csv -- \
    $P > $OUT/probe_sq2.json
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $OUT -o occ --output-format csv -- \
    $P > $OUT/probe_occ.json
echo done $TAG
