#!/bin/bash
out=gpurun_out/${1:-r02cg}; mkdir -p $out
timeout -k 10 300 python -u tools/ab_builds.py --config c4 --reps 10 --rounds 3 base=weightedld_amd/libweightedld.so cg2048=build/exp/cg2048/libweightedld.so > $out/ab_c4.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_builds.py --config c4 --thr 0.005 --reps 6 --rounds 2 "base=weightedld_amd/libweightedld.so@WLD_AB_OPTS=screen=2" "cg2048=build/exp/cg2048/libweightedld.so@WLD_AB_OPTS=screen=2" > $out/ab_c4_thr005_forced.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/shard_sim.py --config c4 --worlds 2,4,8 --reps 5 > $out/shard_sim_c4.txt 2>&1 || exit 1
echo done
