#!/bin/bash
# round-6 GPU call L: stage-top order in the B-rolled screens (in-tree build =
# B roll): A-split (row block 0's A and B block 0 read first, its MFMAs
# waiting only for them), read-first (the next stage's copies issued after
# this stage's reads), both; harness at C4, the 1/8 shard and LD blocks
out=gpurun_out/r06l; mkdir -p $out; export TMPDIR=/tmp
B="base=weightedld_amd/libweightedld.so asplit=build/exp/asplit/libweightedld.so rfirst=build/exp/rfirst/libweightedld.so asrf=build/exp/asrf/libweightedld.so"
tools/gpu_step.sh 400 $out/ab_c4.log python tools/ab_builds.py --config c4 --reps 30 --rounds 3 $B || exit $?
WLD_AB_SHARD=8 tools/gpu_step.sh 300 $out/ab_s8.log python tools/ab_builds.py --config c4 --reps 40 --rounds 3 $B || exit $?
WLD_AB_DATA=ldblocks tools/gpu_step.sh 300 $out/ab_ldb.log python tools/ab_builds.py --config c4 --reps 20 --rounds 3 base=weightedld_amd/libweightedld.so asplit=build/exp/asplit/libweightedld.so || exit $?
echo done
