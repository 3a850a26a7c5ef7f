#!/bin/bash
# Collect the round-N rocprofv3 evidence for profiles/ (run on the GPU box).
#   kernel trace + stats of the bench command, then one --pmc pass per
#   counter group (never combined with tracing), each under its own timeout.
# Usage: tools/profile_round.sh r02 [single|twins]
#   then: python tools/summarize_profile.py gpurun_out/prof_<tag> <tag>
#   (twins: tag r02t, mode twins)
set -e
TAG=${1:-r01}
MODE=${2:-single}
PM=0; [ "$MODE" = twins ] && PM=1
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o trace --output-format csv -- \
    python3 -u bench.py --mode $MODE --no-cpu-baseline > $OUT/bench_under_trace.json
P="python3 -u tools/probe.py --phase solve --reps 1 --mode $PM"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT -o fetch --output-format csv -- $P > $OUT/probe_fetch.json
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT -o write --output-format csv -- $P > $OUT/probe_write.json
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $OUT -o sq1 --output-format csv -- \
    $P > $OUT/probe_sq1.json
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $OUT -o sq2 --output-format csv -- \
    $P > $OUT/probe_sq2.json
# occupancy and LDS-array activity of the same launch (own pass)
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $OUT -o occ --output-format csv -- \
    $P > $OUT/probe_occ.json || echo "occupancy pass failed (counters unavailable?)"
if [ "$MODE" = single ]; then
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT -o fetch_score --output-format csv -- \
      python3 -u tools/probe.py --phase score --reps 1 > $OUT/probe_fetch_score.json
fi
echo done
