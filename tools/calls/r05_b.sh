#!/bin/bash
# round-5 GPU call B: the fp6 x {e2m3, e3m2} dual-reading screen: its tests,
# then A/B against the round-4 fp6 x fp4 kernel at C4
out=gpurun_out/r05b; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 600 $out/tests_fp6.log python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_fp6.py tests/test_gpu_screen.py || exit 1
tools/gpu_step.sh 300 $out/ab_c4.log python3 tools/ab_builds.py --config c4 --reps 10 --rounds 3 \
  old=build/exp/old/libweightedld.so new=weightedld_amd/libweightedld.so || exit 1
echo done
