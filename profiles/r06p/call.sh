#!/bin/bash
# round-6 GPU call P: full-run items (C2) at 7 and 8 workgroups per CU
# (c2w7: 70 VGPRs; c2w8: 64 with 9 spilled); the candidate loop's occupancy
# builds again on LD blocks (nopf5, as5 against the in-tree build)
out=gpurun_out/r06p; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 300 $out/ab_c2.log python tools/ab_builds.py --config c2 --reps 40 --rounds 4 base=weightedld_amd/libweightedld.so c2w7=build/exp/c2w7/libweightedld.so c2w8=build/exp/c2w8/libweightedld.so || exit $?
WLD_AB_DATA=ldblocks tools/gpu_step.sh 400 $out/ab_ldb.log python tools/ab_builds.py --config c4 --reps 20 --rounds 4 base=weightedld_amd/libweightedld.so nopf5=build/exp/nopf5/libweightedld.so as5=build/exp/as5/libweightedld.so as4=build/exp/as4/libweightedld.so || exit $?
echo done
