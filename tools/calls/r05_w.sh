#!/bin/bash
# round-5 GPU call W: the tile-pair fp6 screen at three workgroups per CU
# (6 waves per SIMD, 80 VGPRs, epilogue spills) against two, at C4 and C5
out=gpurun_out/r05w; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 400 $out/ab_c4.log python3 tools/ab_builds.py --config c4 --reps 10 --rounds 3 \
  base=weightedld_amd/libweightedld.so pair6=build/exp/pair6/libweightedld.so || exit 1
tools/gpu_step.sh 400 $out/ab_c5.log python3 tools/ab_builds.py --config c5 --reps 4 --rounds 2 \
  base=weightedld_amd/libweightedld.so pair6=build/exp/pair6/libweightedld.so || exit 1
echo done
