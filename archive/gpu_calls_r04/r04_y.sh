#!/bin/bash
# round-4 GPU call Y: the fp6 screen with 2x2 waves (32 rows x 32 columns
# each: half the B minor-bit masks per wave) against the default at C4; rows
# with fp6 forced; the fp6/screen/parity tests on the variant
out=gpurun_out/r04y; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 400 $out/ab_c4.txt python tools/ab_builds.py --config c4 --reps 20 --rounds 3 \
  base=weightedld_amd/libweightedld.so q=build/exp/f62x2/libweightedld.so || exit $?
tools/gpu_step.sh 200 $out/ab_c4_thr.txt python tools/ab_builds.py --config c4 --thr 0.02 --reps 3 --rounds 1 \
  base=weightedld_amd/libweightedld.so@WLD_AB_OPTS=screen_fp6=2 q=build/exp/f62x2/libweightedld.so@WLD_AB_OPTS=screen_fp6=2 || exit $?
cp build/exp/f62x2/libweightedld.so weightedld_amd/libweightedld.so
tools/gpu_step.sh 600 $out/tests_q.log python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fp6.py tests/test_gpu_screen.py tests/test_gpu_parity.py || exit $?
echo done
