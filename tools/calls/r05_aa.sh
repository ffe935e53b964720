#!/bin/bash
# round-5 GPU call AA: the tile-pair list's XCD super-block side (16 default;
# 4, 8, 32) at C4 and C5; L2 hit rate of the side-8 build
out=gpurun_out/r05aa; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 500 $out/ab_c4.log python3 tools/ab_builds.py --config c4 --reps 10 --rounds 3 \
  base=weightedld_amd/libweightedld.so ks4=build/exp/ks4/libweightedld.so ks8=build/exp/ks8/libweightedld.so \
  ks32=build/exp/ks32/libweightedld.so || exit 1
tools/gpu_step.sh 500 $out/ab_c5.log python3 tools/ab_builds.py --config c5 --reps 4 --rounds 2 \
  base=weightedld_amd/libweightedld.so ks8=build/exp/ks8/libweightedld.so || exit 1
echo done
