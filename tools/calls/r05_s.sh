#!/bin/bash
# round-5 GPU call S: the C2 item kernel with each 16-position group's operands
# formed before its 16 MFMAs (five / four workgroups per CU), and its wave
# timeline; tile pairs vs single tiles at 1/2 and 1/4 shards of C4
out=gpurun_out/r05s; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 400 $out/ab_c2.log python3 tools/ab_builds.py --config c2 --reps 20 --rounds 3 \
  base=weightedld_amd/libweightedld.so pre5=build/exp/i_pre5/libweightedld.so pre4=build/exp/i_pre4/libweightedld.so || exit 1
tools/gpu_step.sh 200 $out/item_trace_pre4.log python3 tools/item_trace.py build/exp/i_pre4_trace/libweightedld.so c2 20 || exit 1
for k in 2 4; do
  tools/gpu_step.sh 300 $out/ab_shard$k.log env WLD_AB_SHARD=$k python3 tools/ab_builds.py --config c4 --reps 10 --rounds 3 \
    pairs=weightedld_amd/libweightedld.so@WLD_AB_OPTS=fp6_pairs_min_tiles=0 \
    single=weightedld_amd/libweightedld.so@WLD_AB_OPTS=fp6_pairs_min_tiles=1000000000 || exit 1
done
echo done
