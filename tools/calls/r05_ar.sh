#!/bin/bash
# round-5 GPU call AR: single tiles against (wide) tile pairs on small lists:
# rank 0's 1/16 shard of C4 (3,064 tiles) and C2 (528 tiles, fp6 forced)
out=gpurun_out/r05ar; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 300 $out/ab_shard16.log env WLD_AB_SHARD=16 python3 tools/ab_builds.py --config c4 --reps 20 --rounds 3 \
  single=weightedld_amd/libweightedld.so pairs=weightedld_amd/libweightedld.so@WLD_AB_OPTS=fp6_pairs_min_tiles=0 || exit 1
tools/gpu_step.sh 300 $out/ab_shard4.log env WLD_AB_SHARD=4 python3 tools/ab_builds.py --config c4 --reps 20 --rounds 3 \
  single=weightedld_amd/libweightedld.so@WLD_AB_OPTS=fp6_pairs_min_tiles=100000 pairs=weightedld_amd/libweightedld.so || exit 1
echo done
