#!/bin/bash
# round-4 GPU call O: the fp6 screen on two tiles of a row per 8-wave
# workgroup (pairs build) against the one-tile kernel at C4; rows with fp6
# forced on LD blocks; then the fp6 and screen tests on the pairs build
out=gpurun_out/r04o; mkdir -p $out; export TMPDIR=/tmp
B="base=weightedld_amd/libweightedld.so pairs=build/exp/pairs/libweightedld.so"
tools/gpu_step.sh 300 $out/ab_c4.txt python tools/ab_builds.py --config c4 --reps 20 --rounds 3 $B || exit $?
tools/gpu_step.sh 200 $out/ab_c4_thr.txt python tools/ab_builds.py --config c4 --thr 0.02 --reps 3 --rounds 1 \
  base=weightedld_amd/libweightedld.so@WLD_AB_OPTS=screen_fp6=2 pairs=build/exp/pairs/libweightedld.so@WLD_AB_OPTS=screen_fp6=2 || exit $?
WLD_AB_DATA=ldblocks WLD_AB_OPTS=screen_fp6=2 tools/gpu_step.sh 300 $out/ab_ld_fp6.txt python tools/ab_builds.py --config c4 --reps 3 --rounds 1 $B || exit $?
cp build/exp/pairs/libweightedld.so weightedld_amd/libweightedld.so
tools/gpu_step.sh 600 $out/tests_pairs.log python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fp6.py tests/test_gpu_screen.py tests/test_gpu_parity.py || exit $?
echo done
