#!/bin/bash
# round-5 GPU session 1: the GPU suite on the round's first source, the
# config-5 solver sweep on the HEAD library, and lone
# large-block probes (n = 2000 singles, 3000-pair twins) as the baseline of
# the large-block work
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5a_tests.log 2>&1 || { tail -30 gpurun_out/r5a_tests.log; exit 1; }
tail -3 gpurun_out/r5a_tests.log
timeout -k 10 120 python tools/probe.py --n 2000 --blocks 1 --phase solve --reps 3 > gpurun_out/r5a_n2000_lone.json || exit 1
cat gpurun_out/r5a_n2000_lone.json | cut -c1-300
timeout -k 10 200 python tools/probe.py --n 2000 --phase solve --reps 2 > gpurun_out/r5a_n2000_round.json || exit 1
cat gpurun_out/r5a_n2000_round.json | cut -c1-300
timeout -k 10 200 python tools/probe.py --mode 1 --n 3000 --phase solve --reps 2 > gpurun_out/r5a_tw3000_round.json || exit 1
cat gpurun_out/r5a_tw3000_round.json | cut -c1-300
timeout -k 10 700 python -u tools/solver_sweep.py > gpurun_out/r05_solver_sweep.jsonl 2> gpurun_out/r5a_sweep.err || { tail gpurun_out/r5a_sweep.err; exit 1; }
wc -l gpurun_out/r05_solver_sweep.jsonl
echo all-done
