#!/bin/bash
# dev sweep: phase timings of the block kernel designs on several rounds
cd $GRAFT_REPO_ROOT
for args in "$@"; do
  echo "ARGS $args"
  timeout -k 10 120 python -u tools/probe.py --reps 2 $args 2>&1 | grep -v amdgpu.ids || exit 1
done
