#!/bin/bash
# round-6 GPU call K: two B slots rolled through each stage (block n + 2's
# LDS read issued once block n's masked MFMAs are issued, in flight under
# block n + 1's) in the fp6 and i8 screens, A/B against the tree's build:
# harness at C4, LD blocks and rank 0's 1/8 shard, then bench.py lines
out=gpurun_out/r06k; mkdir -p $out; export TMPDIR=/tmp
B="cur=weightedld_amd/libweightedld.so broll=build/exp/broll/libweightedld.so"
tools/gpu_step.sh 300 $out/ab_c4.log python tools/ab_builds.py --config c4 --reps 30 --rounds 3 $B || exit $?
WLD_AB_DATA=ldblocks tools/gpu_step.sh 300 $out/ab_ldb.log python tools/ab_builds.py --config c4 --reps 20 --rounds 3 $B || exit $?
WLD_AB_SHARD=8 tools/gpu_step.sh 200 $out/ab_s8.log python tools/ab_builds.py --config c4 --reps 40 --rounds 3 $B || exit $?
for i in 1 2; do
  tools/gpu_step.sh 200 $out/c4_cur_$i.log python bench.py --no-cpu-baseline || exit $?
  WLD_LIB_PATH=build/exp/broll/libweightedld.so tools/gpu_step.sh 200 $out/c4_broll_$i.log python bench.py --no-cpu-baseline || exit $?
  tools/gpu_step.sh 200 $out/ldb_cur_$i.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
  WLD_LIB_PATH=build/exp/broll/libweightedld.so tools/gpu_step.sh 200 $out/ldb_broll_$i.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
done
echo done
