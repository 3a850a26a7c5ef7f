#!/bin/bash
# Round-end evidence on the current source (GPU box), in three calls (each
# fits one gpurun limit):
#   phase 1: the GPU test suite, smoke(), rocprofv3 profiles of the full round
#            (tag $TAG) and the twins round ($TAG"t");
#   phase 1b: rank 0's shard at N = 8, 4, 2 ($TAG"s8/s4/s2"), the reference's
#            own block sizes ($TAG"n": 477 x n = 2000, $TAG"w": 6 x 3000 pairs);
#            then locally: python tools/summarize_profile.py gpurun_out/prof_<tag> <tag>
#   phase 2: bench lines for every mode (they read the committed summaries), shard probes
cd "$(dirname "$0")/.." || exit 2
TAG=${2:-r03b}
case ${1:-1} in
  1)
    bash tools/gpu_run.sh tests smoke > gpurun_out/final_ts.log 2>&1 || exit 1
    grep -q " passed" gpurun_out/tests.log && ! grep -q " failed" gpurun_out/tests.log || exit 1
    bash tools/profile_round.sh $TAG single > gpurun_out/prof_$TAG.log 2>&1 || exit 1
    bash tools/profile_round.sh ${TAG}t twins > gpurun_out/prof_${TAG}t.log 2>&1 || exit 1
    ;;
  1b)
    bash tools/profile_shards.sh ${TAG}s || exit 1
    # the reference's own block sizes: 477 blocks of n = 2000, 6 of 3000 pairs
    bash tools/profile_shard.sh ${TAG}n 477 "--n 2000" > gpurun_out/prof_${TAG}n.log 2>&1 || exit 1
    bash tools/profile_shard.sh ${TAG}w 6 "--mode 1 --n 3000" > gpurun_out/prof_${TAG}w.log 2>&1 || exit 1
    ;;
  2)
    bash tools/gpu_run.sh bench bench_twins bench_triplets bench_n2000cpu bench_twins3000 > gpurun_out/final_bench.log 2>&1 || exit 1
    bash tools/shard_probe.sh > gpurun_out/shard_probe.log 2>&1 || exit 1
    ;;
esac
echo final-done
