#!/bin/bash
# round-4 GPU call R: the fp6 screen with its epilogue in the MFMA shadow
# (persistent workgroups, pipe build) against the one-tile kernel at C4;
# rows with fp6 forced; then the fp6/screen/parity tests on the pipe build
out=gpurun_out/r04r; mkdir -p $out; export TMPDIR=/tmp
B="base=weightedld_amd/libweightedld.so pipe=build/exp/pipe/libweightedld.so"
tools/gpu_step.sh 300 $out/ab_c4.txt python tools/ab_builds.py --config c4 --reps 20 --rounds 3 $B || exit $?
tools/gpu_step.sh 200 $out/ab_c4_thr.txt python tools/ab_builds.py --config c4 --thr 0.02 --reps 3 --rounds 1 \
  base=weightedld_amd/libweightedld.so@WLD_AB_OPTS=screen_fp6=2 pipe=build/exp/pipe/libweightedld.so@WLD_AB_OPTS=screen_fp6=2 || exit $?
cp build/exp/pipe/libweightedld.so weightedld_amd/libweightedld.so
tools/gpu_step.sh 600 $out/tests_pipe.log python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fp6.py tests/test_gpu_screen.py tests/test_gpu_parity.py || exit $?
echo done
