#!/bin/bash
# round-5 GPU call H: fp6 screen on tile pairs (one A image for two column
# tiles, 8-wave workgroups) with fp4 / 6-bit B, against single tiles and the
# round-4 kernel; fp6 row tests on the default (pairs, fp4 B)
out=gpurun_out/r05h; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 400 $out/tests_fp6.log python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_fp6.py tests/test_gpu_screen.py -k "not full_size" || exit 1
tools/gpu_step.sh 500 $out/ab_c4.log python3 tools/ab_builds.py --config c4 --reps 10 --rounds 3 \
  old=build/exp/old/libweightedld.so pairs_b4=weightedld_amd/libweightedld.so pairs_b6=build/exp/pairs_b6/libweightedld.so \
  single_b4=build/exp/single_b4/libweightedld.so single_b6=build/exp/single_b6/libweightedld.so || exit 1
echo done
