#!/bin/bash
# round-6 GPU call AG: the screens' all-valid epilogue with a sufficient test
# first (largest numerator against the smallest marginal, 2^-10 margin; the
# exact per-pair form only when it fails) against the exact form alone: fp6,
# i8 and screen tests on it, then A/B at C4, the 1/8 shard, LD blocks
out=gpurun_out/r06ag; mkdir -p $out; export TMPDIR=/tmp
WLD_LIB_PATH=build/exp/epis/libweightedld.so tools/gpu_step.sh 700 $out/tests.log python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fp6.py tests/test_gpu_i8pairs.py tests/test_gpu_screen.py -m gpu || exit $?
B="base=weightedld_amd/libweightedld.so epis=build/exp/epis/libweightedld.so"
tools/gpu_step.sh 300 $out/ab_c4.log python tools/ab_builds.py --config c4 --reps 30 --rounds 4 $B || exit $?
WLD_AB_SHARD=8 tools/gpu_step.sh 300 $out/ab_s8.log python tools/ab_builds.py --config c4 --reps 40 --rounds 3 $B || exit $?
WLD_AB_DATA=ldblocks tools/gpu_step.sh 300 $out/ab_ldb.log python tools/ab_builds.py --config c4 --reps 20 --rounds 3 $B || exit $?
echo done
