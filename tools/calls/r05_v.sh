#!/bin/bash
# round-5 GPU call V: the item kernel without the stage prefetch (70 VGPRs) at
# six, seven, eight workgroups per CU, at C2 and on C4 LD blocks; timeline
out=gpurun_out/r05v; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 400 $out/ab_c2.log python3 tools/ab_builds.py --config c2 --reps 20 --rounds 3 \
  base=weightedld_amd/libweightedld.so nopf6=build/exp/i_nopf6/libweightedld.so nopf7=build/exp/i_nopf7/libweightedld.so \
  nopf8=build/exp/i_nopf8/libweightedld.so || exit 1
tools/gpu_step.sh 400 $out/ab_ldb.log env WLD_AB_DATA=ldblocks python3 tools/ab_builds.py --config c4 --reps 10 --rounds 2 \
  base=weightedld_amd/libweightedld.so nopf7=build/exp/i_nopf7/libweightedld.so || exit 1
tools/gpu_step.sh 200 $out/item_trace_nopf7.log python3 tools/item_trace.py build/exp/i_nopf7_trace/libweightedld.so c2 20 $out/item_trace_nopf7.npy || exit 1
echo done
