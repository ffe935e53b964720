#!/bin/bash
# Screen policy calibration at C4: pair phase with the screen always (2), never (0)
# and auto (1) at thresholds where many tiles are candidates; then the screen tests.
out=gpurun_out/${1:-r02sp}; mkdir -p $out
lib=weightedld_amd/libweightedld.so
for thr in 0.001 0.003 0.005 0.01; do
  timeout -k 10 300 python -u tools/ab_builds.py --config c4 --thr $thr --reps 6 --rounds 1 \
    "always=$lib@WLD_AB_OPTS=screen=2" "never=$lib@WLD_AB_OPTS=screen=0" "auto=$lib@WLD_AB_OPTS=screen=1" > $out/policy_$thr.txt 2>&1 || exit 1
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_screen.py -x -q --timeout 200 --timeout-method thread > $out/screen_tests.txt 2>&1 || exit 1
echo done
