#!/bin/bash
# A/B of experimental builds at C4 (Henikoff and unit weights) + the screen tests on the variant.
#   tools/calls/r02_ab.sh TAG VARIANT...   (build/exp/VARIANT/libweightedld.so)
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
builds="base=weightedld_amd/libweightedld.so"
for v in "$@"; do builds="$builds $v=build/exp/$v/libweightedld.so"; done
timeout -k 10 400 python -u tools/ab_builds.py --config c4 --reps 10 --rounds 3 $builds > $out/ab_c4.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_builds.py --config c4 --reps 10 --rounds 2 --unweighted $builds > $out/ab_c4_unw.txt 2>&1 || exit 1
for v in "$@"; do
  WLD_TEST_BUILD=build/exp/$v timeout -k 10 300 python -u -m pytest tests/test_gpu_screen.py -x -q --timeout 120 --timeout-method thread > $out/screen_tests_$v.txt 2>&1 || exit 1
done
echo done
