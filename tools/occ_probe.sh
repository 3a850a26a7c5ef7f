cd $GRAFT_REPO_ROOT
for b in 256 1024 2048 2560 3072 3730; do timeout -k 10 120 python -u tools/probe.py --phase solve --reps 3 --blocks $b --flags 128; done > gpurun_out/occ.jsonl 2>&1
for b in 1024 2048 3730; do timeout -k 10 120 python -u tools/probe.py --phase solve --reps 3 --blocks $b --flags 128 --state-round 10; done >> gpurun_out/occ.jsonl 2>&1
