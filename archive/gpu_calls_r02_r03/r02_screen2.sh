#!/bin/bash
# Two-plane screen: screen tests, then the C4 pair phase with the screen never
# (0), one-plane (2), two-plane (3) and auto (1) at low thresholds.
out=gpurun_out/${1:-r02s2}; mkdir -p $out
export TMPDIR=/tmp
lib=weightedld_amd/libweightedld.so
tools/gpu_step.sh 400 $out/screen_tests.txt python -u -m pytest tests/test_gpu_screen.py -v -s --timeout 200 --timeout-method thread || exit $?
for thr in 0.005 0.01 0.02 0.03; do
  timeout -k 10 300 python -u tools/ab_builds.py --config c4 --thr $thr --reps 6 --rounds 1 \
    "never=$lib@WLD_AB_OPTS=screen=0" "one=$lib@WLD_AB_OPTS=screen=2" "two=$lib@WLD_AB_OPTS=screen=3" \
    "auto=$lib@WLD_AB_OPTS=screen=1" > $out/ab_$thr.txt 2>&1 || exit 1
done
echo done
