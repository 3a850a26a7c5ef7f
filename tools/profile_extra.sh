#!/bin/bash
# rocprofv3 evidence for config 5 and the triplet extension:
# lsap_i64_kernel on n = 256 x 65536 hashed instances (kernel trace + SQ and
# occupancy PMC passes, each its own run) and the triplets launch (6 blocks of
# 256 units, tools/profile_shard.sh).  Then locally:
#   python tools/summarize_profile.py gpurun_out/prof_<tag>l <tag>l ; ... <tag>tr
set -e
TAG=${1:-r05}
OUT=gpurun_out/prof_${TAG}l
mkdir -p $OUT
export TMPDIR=/tmp
P="python3 -u tools/lsap_time.py 256x65536"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o trace --output-format csv -- $P > $OUT/lsap_trace.json
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT -o fetch --output-format csv -- $P > $OUT/lsap_fetch.json
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $OUT -o sq1 --output-format csv -- \
    $P > $OUT/lsap_sq1.json
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $OUT -o sq2 --output-format csv -- \
    $P > $OUT/lsap_sq2.json
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $OUT -o occ --output-format csv -- \
    $P > $OUT/lsap_occ.json
bash tools/profile_shard.sh ${TAG}tr 6 "--mode 2" > gpurun_out/prof_${TAG}tr.log 2>&1
echo done
