#!/bin/bash
# PMC passes over one round-0 solve launch (tile + sparse kernels), dev tool:
#   tools/tile_pmc.sh <outdir>
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
OUT=${1:-gpurun_out/tpmc}; mkdir -p $OUT
P="python3 -u tools/probe.py --phase solve --reps 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $OUT -o sq1 --output-format csv -- $P > $OUT/p1.json &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $OUT -o sq2 --output-format csv -- $P > $OUT/p2.json &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT -o fetch --output-format csv -- $P > $OUT/p3.json && echo ok
