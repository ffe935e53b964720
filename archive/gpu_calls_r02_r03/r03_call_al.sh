#!/bin/bash
# round-3 GPU call AL: (1) the GPU suite on the default build (the fused scan's
# ticket set fixed for dealt-first workgroups); (2) screen/ref-sums tests on a
# build that splits candidate tiles with more than 8 sub-blocks into two work
# items by a-row halves (WLD_CAND_SPLIT); (3) A/B on LD blocks
out=gpurun_out/r03al; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 900 $out/gpu_tests.txt python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread || exit $?
grep -q " passed" $out/gpu_tests.txt && ! grep -q " failed" $out/gpu_tests.txt || { echo "suite not green"; exit 1; }
WLD_TEST_BUILD=build/exp/split tools/gpu_step.sh 600 $out/tests_split.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_screen.py tests/test_gpu_refsums.py -m gpu -k "not full" || exit $?
grep -q " passed" $out/tests_split.log && ! grep -q " failed" $out/tests_split.log || { echo "split tests not green"; exit 1; }
B="nosplit=build/exp/nosplit/libweightedld.so split=build/exp/split/libweightedld.so"
WLD_AB_DATA=ldblocks timeout -k 10 400 python tools/ab_builds.py --config c4 --reps 10 --rounds 3 $B > $out/ab_ldb.txt 2>&1 || { echo "ab ldb failed $?"; exit 1; }
timeout -k 10 400 python tools/ab_builds.py --config c4 --thr 0.02 --reps 10 --rounds 2 $B > $out/ab_c4_thr002.txt 2>&1 || { echo "ab c4 0.02 failed $?"; exit 1; }
echo done
