#!/bin/bash
# round-5 GPU call C: fp6 screen with A straight to registers (default) vs A
# through LDS vs the round-4 fp6 x fp4 kernel; fp6 row tests on the default
out=gpurun_out/r05c; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 400 $out/ab_c4.log python3 tools/ab_builds.py --config c4 --reps 10 --rounds 3 \
  old=build/exp/old/libweightedld.so alds=build/exp/alds/libweightedld.so areg=weightedld_amd/libweightedld.so || exit 1
tools/gpu_step.sh 400 $out/tests_fp6.log python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_fp6.py -k "not full_size" || exit 1
tools/gpu_step.sh 300 $out/bench_c4.log python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
echo done
