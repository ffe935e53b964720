#!/bin/bash
# round-6 GPU call AH: s_setprio 1 around each stage's MFMA cluster of the fp6
# screen (0 for the barrier, copies and epilogue) against none: A/B at C4 and
# the 1/8 shard
out=gpurun_out/r06ah; mkdir -p $out; export TMPDIR=/tmp
B="base=weightedld_amd/libweightedld.so prio=build/exp/prio/libweightedld.so"
tools/gpu_step.sh 300 $out/ab_c4.log python tools/ab_builds.py --config c4 --reps 30 --rounds 5 $B || exit $?
WLD_AB_SHARD=8 tools/gpu_step.sh 300 $out/ab_s8.log python tools/ab_builds.py --config c4 --reps 40 --rounds 3 $B || exit $?
echo done
