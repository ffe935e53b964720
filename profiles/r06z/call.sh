#!/bin/bash
# round-6 GPU call Z (diagnostic): the fp6 screen with its stage loop run
# 1x / 2x / 3x over the same operands (same entries, epilogues and launch;
# KREP x the MFMA work): the per-entry overhead is T(1) - (T(2) - T(1)).
# C4 and the 1/8 shard
out=gpurun_out/r06z; mkdir -p $out; export TMPDIR=/tmp
B="k1=build/exp/krep1/libweightedld.so k2=build/exp/krep2/libweightedld.so k3=build/exp/krep3/libweightedld.so"
tools/gpu_step.sh 300 $out/ab_c4.log python tools/ab_builds.py --config c4 --reps 20 --rounds 3 $B || exit $?
WLD_AB_SHARD=8 tools/gpu_step.sh 300 $out/ab_s8.log python tools/ab_builds.py --config c4 --reps 40 --rounds 3 $B || exit $?
echo done
