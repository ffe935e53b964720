#!/bin/bash
# round-4 GPU call N: fp6 screen with A loaded straight into registers
# (areg3, three workgroups per CU) against the default and wg3 at C4; row
# counts at a threshold with candidates and on LD blocks
out=gpurun_out/r04n; mkdir -p $out; export TMPDIR=/tmp
B="base=weightedld_amd/libweightedld.so areg3=build/exp/areg3/libweightedld.so wg3=build/exp/wg3/libweightedld.so"
tools/gpu_step.sh 400 $out/ab_c4.txt python tools/ab_builds.py --config c4 --reps 20 --rounds 3 $B || exit $?
tools/gpu_step.sh 200 $out/ab_c4_thr.txt python tools/ab_builds.py --config c4 --thr 0.05 --reps 3 --rounds 1 $B || exit $?
WLD_AB_DATA=ldblocks tools/gpu_step.sh 300 $out/ab_ld.txt python tools/ab_builds.py --config c4 --reps 10 --rounds 2 $B || exit $?
echo done
