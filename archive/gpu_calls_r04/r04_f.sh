#!/bin/bash
# round-4 GPU call F: fp6 screen with optional several tiles per workgroup
# (WLD_FP6_TPW) and 3 vs 4 waves (WLD_FP6_WG); the gather enqueued behind the
# scan (WLD_SPEC_GATHER); the item kernel's tail loads: tests, C4 and C2 A/B,
# bench lines
out=gpurun_out/r04f; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 60 $out/fp6_32_probe.txt tools/probes/fp6_32_probe || exit $?
tools/gpu_step.sh 600 $out/tests.txt python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fp6.py tests/test_gpu_refsums.py tests/test_gpu_parity.py \
  -k "fp6 or gather_behind or staging_overflow or ref_rows_bit_exact or ref_dense" || exit $?
tools/gpu_step.sh 400 $out/ab_c4.txt python tools/ab_builds.py --config c4 --reps 20 --rounds 3 \
  base=weightedld_amd/libweightedld.so tpw2=build/exp/tpw2/libweightedld.so tpw4=build/exp/tpw4/libweightedld.so \
  wg3=build/exp/wg3/libweightedld.so nbuf3=build/exp/nbuf3/libweightedld.so nodma=build/exp/nodma/libweightedld.so fp632=build/exp/fp632/libweightedld.so || exit $?
tools/gpu_step.sh 300 $out/ab_c2.txt python tools/ab_builds.py --config c2 --reps 30 --rounds 3 \
  spec=weightedld_amd/libweightedld.so nospec=build/exp/nospec/libweightedld.so tailold=build/exp/tailold/libweightedld.so \
  noepi=build/exp/noepi/libweightedld.so noload=build/exp/noload/libweightedld.so nosel=build/exp/nosel/libweightedld.so \
  cvt=build/exp/cvt/libweightedld.so || exit $?
WLD_AB_DATA=ldblocks tools/gpu_step.sh 300 $out/ab_ldb.txt python tools/ab_builds.py --config c4 --reps 10 --rounds 3 \
  base=weightedld_amd/libweightedld.so cvt=build/exp/cvt/libweightedld.so || exit $?
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c2.log python bench.py --config c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
echo done
