#!/bin/bash
# rank 0's shard at N = 8, 4, 2 (tools/profile_shard.sh), one after another.
set -e
TAG=${1:-r03s}
bash tools/profile_shard.sh ${TAG}8 467 > gpurun_out/prof_${TAG}8.log 2>&1
bash tools/profile_shard.sh ${TAG}4 933 > gpurun_out/prof_${TAG}4.log 2>&1
bash tools/profile_shard.sh ${TAG}2 1865 > gpurun_out/prof_${TAG}2.log 2>&1
echo done
