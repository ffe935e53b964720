#!/bin/bash
# round-6 GPU call U: LDS-staged candidate items at 5 workgroups per CU, the
# launch's grid 1,024 (lds5) against 768 and 896, and HEAD; LD blocks
out=gpurun_out/r06u; mkdir -p $out; export TMPDIR=/tmp
B="head=build/exp/head/libweightedld.so lds5=build/exp/lds5/libweightedld.so g768=build/exp/lds5g768/libweightedld.so g896=build/exp/lds5g896/libweightedld.so"
WLD_AB_DATA=ldblocks tools/gpu_step.sh 300 $out/ab_ldb.log python tools/ab_builds.py --config c4 --reps 20 --rounds 4 $B || exit $?
echo done
