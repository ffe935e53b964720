#!/bin/bash
# round-5 GPU call L: the epilogue's quotients by T from an f64 reciprocal
# (default) vs eight IEEE f32 divisions: bit-exact tests (dense stats, rows),
# then A/B at C2 (every pair through the epilogue) and on LD blocks
out=gpurun_out/r05l; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 600 $out/tests.log python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_refsums.py tests/test_gpu_screen.py -k "not full_bench and not c5_ldblocks" || exit 1
tools/gpu_step.sh 400 $out/ab_c2.log python3 tools/ab_builds.py --config c2 --reps 20 --rounds 3 \
  ieeediv=build/exp/ieeediv/libweightedld.so divt=weightedld_amd/libweightedld.so || exit 1
WLD_AB_DATA=ldblocks tools/gpu_step.sh 400 $out/ab_ldb.log python3 tools/ab_builds.py --config c4 --reps 10 --rounds 2 \
  ieeediv=build/exp/ieeediv/libweightedld.so divt=weightedld_amd/libweightedld.so || exit 1
echo done
