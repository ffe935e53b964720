#!/bin/bash
# round-5 GPU call AQ: the wide-wave tile-pair screen as the default build:
# fp6 and screen tests (tile pairs now also forced at small sizes), then rank
# 0's 1/8 shard on single tiles (default under 8,192 tiles) against tile pairs
# forced, and the 1/2 shard wide against the eight-wave kernel
out=gpurun_out/r05aq; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 400 $out/tests.log python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_fp6.py tests/test_gpu_screen.py -m gpu || exit 1
grep -q " passed" $out/tests.log && ! grep -q "failed\|error" $out/tests.log || { echo "tests not green"; exit 1; }
tools/gpu_step.sh 300 $out/ab_shard8.log env WLD_AB_SHARD=8 python3 tools/ab_builds.py --config c4 --reps 20 --rounds 3 \
  single=weightedld_amd/libweightedld.so pairs=weightedld_amd/libweightedld.so@WLD_AB_OPTS=fp6_pairs_min_tiles=0 || exit 1
tools/gpu_step.sh 300 $out/ab_shard2.log env WLD_AB_SHARD=2 python3 tools/ab_builds.py --config c4 --reps 20 --rounds 3 \
  wide=weightedld_amd/libweightedld.so narrow=build/exp/narrow/libweightedld.so || exit 1
echo done
