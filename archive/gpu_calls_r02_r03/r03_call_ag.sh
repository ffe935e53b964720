#!/bin/bash
# round-3 GPU call AG: the two-wave screen (32 a rows x 64 b columns per wave,
# pair_screen_wide_kernel, -DWLD_SCR_WIDE): screen/ref-sums bit-identity tests
# on that build, then A/B against the four-wave screen at C4, C5, LD blocks
out=gpurun_out/r03ag; mkdir -p $out; export TMPDIR=/tmp
WLD_TEST_BUILD=build/exp/wide4 tools/gpu_step.sh 600 $out/tests_wide4.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_screen.py tests/test_gpu_refsums.py -m gpu -k "not full" || exit $?
grep -q " passed" $out/tests_wide4.log && ! grep -q "failed" $out/tests_wide4.log || { echo "wide4 tests not green"; exit 1; }
B="base=build/exp/base/libweightedld.so wide4=build/exp/wide4/libweightedld.so wide2=build/exp/wide2/libweightedld.so"
timeout -k 10 400 python tools/ab_builds.py --config c4 --reps 20 --rounds 3 $B > $out/ab_c4.txt 2>&1 || { echo "ab c4 failed $?"; exit 1; }
timeout -k 10 400 python tools/ab_builds.py --config c5 --reps 5 --rounds 2 $B > $out/ab_c5.txt 2>&1 || { echo "ab c5 failed $?"; exit 1; }
WLD_AB_DATA=ldblocks timeout -k 10 400 python tools/ab_builds.py --config c4 --reps 10 --rounds 2 $B > $out/ab_ldb.txt 2>&1 || { echo "ab ldb failed $?"; exit 1; }
timeout -k 10 400 python tools/ab_builds.py --config c4 --unweighted --reps 10 --rounds 2 $B > $out/ab_unw.txt 2>&1 || { echo "ab unw failed $?"; exit 1; }
echo done
