#!/bin/bash
# dev: GPU tests then sparse-kernel probes (full round / N=8 shard, rounds 0 and 10)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -3 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
tools/sweep_probe.sh "--phase solve" "--phase solve --state-round 10" "--blocks 466 --phase solve" "--blocks 466 --phase solve --state-round 10" "$@"
