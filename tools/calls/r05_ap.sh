#!/bin/bash
# round-5 GPU call AP: wide-wave tile-pair fp6 screen (WLD_F6_WIDE: four
# waves of 32 x 64, three workgroups per CU):
# fp6 parity tests on the variant, then A/B against the default at C4, C4 thr
# 0.01 with fp6 forced (rows), C5 and rank 0's 1/4 shard
out=gpurun_out/r05ap; mkdir -p $out; export TMPDIR=/tmp
v=build/exp/wide/libweightedld.so
WLD_LIB_PATH=$v tools/gpu_step.sh 300 $out/tests_fp6.log python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_fp6.py -m gpu || exit 1
grep -q " passed" $out/tests_fp6.log && ! grep -q "failed\|error" $out/tests_fp6.log || { echo "fp6 tests not green"; exit 1; }
tools/gpu_step.sh 400 $out/ab_c4.log python3 tools/ab_builds.py --config c4 --reps 10 --rounds 3 \
  base=weightedld_amd/libweightedld.so wide=$v || exit 1
tools/gpu_step.sh 300 $out/ab_c4_thr01.log python3 tools/ab_builds.py --config c4 --thr 0.01 --reps 3 --rounds 1 \
  base=weightedld_amd/libweightedld.so@WLD_AB_OPTS=screen_fp6=2 wide=$v@WLD_AB_OPTS=screen_fp6=2 || exit 1
tools/gpu_step.sh 400 $out/ab_c5.log python3 tools/ab_builds.py --config c5 --reps 4 --rounds 2 \
  base=weightedld_amd/libweightedld.so wide=$v || exit 1
tools/gpu_step.sh 300 $out/ab_shard4.log env WLD_AB_SHARD=4 python3 tools/ab_builds.py --config c4 --reps 20 --rounds 3 \
  base=weightedld_amd/libweightedld.so wide=$v || exit 1
echo done
