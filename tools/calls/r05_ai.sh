#!/bin/bash
# round-5 GPU call AI: full-run items reading the b operands from f32 planes
# (no converts) against no sharing at all, at six / seven workgroups per CU and
# with the stage's plane loads before the barrier (five per CU); the suites
out=gpurun_out/r05ai; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 400 $out/ab_c2.log python3 tools/ab_builds.py --config c2 --reps 20 --rounds 3 \
  noshare=build/exp/ash0/libweightedld.so planes6=weightedld_amd/libweightedld.so planes7=build/exp/jit7/libweightedld.so \
  bpre5=build/exp/bpre5/libweightedld.so || exit 1
tools/gpu_step.sh 900 $out/tests.log python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_refsums.py tests/test_gpu_parity.py tests/test_gpu_screen.py -k "not full_bench and not c5_ldblocks" || exit 1
tools/gpu_step.sh 200 $out/bench_c2.log python bench.py --config c2 --no-cpu-baseline || exit $?
echo done
