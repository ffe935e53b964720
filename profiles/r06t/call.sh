#!/bin/bash
# round-6 GPU call T: LDS-staged candidate items at 5 workgroups per CU with
# the launch's 1,024 workgroups (lds5) or 1,280 (lds5g, every slot), against
# HEAD, LD blocks, five rounds
out=gpurun_out/r06t; mkdir -p $out; export TMPDIR=/tmp
B="head=build/exp/head/libweightedld.so lds5=build/exp/lds5/libweightedld.so lds5g=build/exp/lds5g/libweightedld.so"
WLD_AB_DATA=ldblocks tools/gpu_step.sh 300 $out/ab_ldb.log python tools/ab_builds.py --config c4 --reps 20 --rounds 5 $B || exit $?
echo done
