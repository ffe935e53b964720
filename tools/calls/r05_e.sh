#!/bin/bash
# round-5 GPU call E: fp6 screen variants at C4 (one-at-a-time harness):
# A through LDS / registers, next stage issued at the stage top / after the
# MFMAs, and two no-epilogue diagnostic builds (timing only, rows wrong)
out=gpurun_out/r05e; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 500 $out/ab_c4.log python3 tools/ab_builds.py --config c4 --reps 10 --rounds 3 \
  old=build/exp/old/libweightedld.so alds_top=build/exp/alds_top/libweightedld.so \
  alds_late=build/exp/alds_late/libweightedld.so areg_top=build/exp/areg_top/libweightedld.so \
  areg_late=weightedld_amd/libweightedld.so noepi_late=build/exp/noepi_late/libweightedld.so \
  noepi_alds_top=build/exp/noepi_alds_top/libweightedld.so || exit 1
echo done
