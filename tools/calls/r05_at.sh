#!/bin/bash
# round-5 GPU call AT: XCD super-block side of the tile-pair list with the
# wide-wave screen (default 16 at C4) against 8 and 32, C4 and the 1/8 shard
out=gpurun_out/r05at; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 400 $out/ab_c4.log python3 tools/ab_builds.py --config c4 --reps 10 --rounds 3 \
  ks16=weightedld_amd/libweightedld.so ks8=build/exp/ks8/libweightedld.so ks32=build/exp/ks32/libweightedld.so || exit 1
tools/gpu_step.sh 300 $out/ab_shard8.log env WLD_AB_SHARD=8 python3 tools/ab_builds.py --config c4 --reps 20 --rounds 3 \
  ks16=weightedld_amd/libweightedld.so ks8=build/exp/ks8/libweightedld.so ks32=build/exp/ks32/libweightedld.so || exit 1
echo done
