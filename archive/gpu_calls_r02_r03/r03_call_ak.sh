#!/bin/bash
# round-3 GPU call AK: the lib.rs-order candidate launch deals each CU's three
# first tiles as a heavy, a light and a middle one (WLD_CAND_MIX) instead of
# three of the heaviest: screen/ref-sums tests on that build, then A/B on LD
# blocks (candidates) and random C4 (none)
out=gpurun_out/r03ak; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 600 $out/tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_screen.py tests/test_gpu_refsums.py -m gpu -k "not full" || exit $?
grep -q " passed" $out/tests.log && ! grep -q " failed" $out/tests.log || { echo "tests not green"; exit 1; }
B="nomix=build/exp/nomix/libweightedld.so mix=build/exp/mix/libweightedld.so"
WLD_AB_DATA=ldblocks timeout -k 10 400 python tools/ab_builds.py --config c4 --reps 10 --rounds 3 $B > $out/ab_ldb.txt 2>&1 || { echo "ab ldb failed $?"; exit 1; }
WLD_AB_DATA=ldblocks timeout -k 10 400 python tools/ab_builds.py --config c4 --thr 0.02 --reps 10 --rounds 2 $B > $out/ab_ldb_thr002.txt 2>&1 || { echo "ab ldb 0.02 failed $?"; exit 1; }
timeout -k 10 400 python tools/ab_builds.py --config c4 --thr 0.02 --reps 10 --rounds 2 $B > $out/ab_c4_thr002.txt 2>&1 || { echo "ab c4 0.02 failed $?"; exit 1; }
echo done
