#!/bin/bash
# round-4 GPU call W: XCD super-block side 8 / 32 tiles against the default
# (16 at C4) for the fp6 screen (C4) and the i8 screen (LD blocks); the full
# run's item kernel at four instead of five workgroups per CU (C2)
out=gpurun_out/r04w; mkdir -p $out; export TMPDIR=/tmp
B="base=weightedld_amd/libweightedld.so xs8=build/exp/xs8/libweightedld.so xs32=build/exp/xs32/libweightedld.so"
tools/gpu_step.sh 400 $out/ab_c4.txt python tools/ab_builds.py --config c4 --reps 15 --rounds 3 $B || exit $?
WLD_AB_DATA=ldblocks tools/gpu_step.sh 400 $out/ab_ld.txt python tools/ab_builds.py --config c4 --reps 10 --rounds 2 $B || exit $?
tools/gpu_step.sh 300 $out/ab_c2.txt python tools/ab_builds.py --config c2 --reps 30 --rounds 3 \
  base=weightedld_amd/libweightedld.so iwg4=build/exp/iwg4/libweightedld.so || exit $?
echo done
