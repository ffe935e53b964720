#!/bin/bash
# round-4 GPU call S: the one-plane i8 screen with its epilogue in the MFMA
# shadow (i8pipe build) on LD blocks (the i8 screen's workload) against the
# default; rows; then the screen and parity tests on the i8pipe build
out=gpurun_out/r04s; mkdir -p $out; export TMPDIR=/tmp
B="base=weightedld_amd/libweightedld.so i8pipe=build/exp/i8pipe/libweightedld.so"
WLD_AB_DATA=ldblocks WLD_AB_OPTS=screen_fp6=0 tools/gpu_step.sh 400 $out/ab_ld.txt python tools/ab_builds.py --config c4 --reps 15 --rounds 2 $B || exit $?
WLD_AB_OPTS=screen_fp6=0 tools/gpu_step.sh 300 $out/ab_c4_i8.txt python tools/ab_builds.py --config c4 --reps 15 --rounds 2 $B || exit $?
cp build/exp/i8pipe/libweightedld.so weightedld_amd/libweightedld.so
tools/gpu_step.sh 600 $out/tests_i8pipe.log python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_screen.py tests/test_gpu_parity.py tests/test_gpu_refsums.py || exit $?
echo done
