#!/bin/bash
# dev: texture-addresser / texture-data busy of the full-round launch (is the
# tile build's row-per-thread wishlist gather TA-bound?)  One pass per block pair.
cd "$(dirname "$0")/.." || exit 2
OUT=gpurun_out/ta_probe; mkdir -p $OUT; export TMPDIR=/tmp
P="python3 -u tools/probe.py --phase solve --reps 1"
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS GRBM_GUI_ACTIVE -d $OUT -o ta --output-format csv -- $P > $OUT/p1.json || exit 1
timeout -s KILL 120 rocprofv3 --pmc TD_TD_BUSY TCP_TOTAL_CACHE_ACCESSES GRBM_GUI_ACTIVE -d $OUT -o td --output-format csv -- $P > $OUT/p2.json || exit 1
echo done
