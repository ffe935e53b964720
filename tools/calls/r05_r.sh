#!/bin/bash
# round-5 GPU call R: the tile-pair fp6 screen with three stage buffers (two
# stages in flight) against the default two, at C4 (and rows at thr 0.01 with
# fp6 forced), at C5, and on rank 0's 1/8 shard
out=gpurun_out/r05r; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 300 $out/tests_guard.log python3 -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_screen.py -k guard || exit 1
tools/gpu_step.sh 400 $out/ab_c4.log python3 tools/ab_builds.py --config c4 --reps 10 --rounds 3 \
  base=weightedld_amd/libweightedld.so ring3=build/exp/ring3/libweightedld.so || exit 1
tools/gpu_step.sh 300 $out/ab_c4_thr01.log python3 tools/ab_builds.py --config c4 --thr 0.01 --reps 3 --rounds 1 \
  base=weightedld_amd/libweightedld.so@WLD_AB_OPTS=screen_fp6=2 ring3=build/exp/ring3/libweightedld.so@WLD_AB_OPTS=screen_fp6=2 || exit 1
tools/gpu_step.sh 400 $out/ab_c5.log python3 tools/ab_builds.py --config c5 --reps 4 --rounds 2 \
  base=weightedld_amd/libweightedld.so ring3=build/exp/ring3/libweightedld.so || exit 1
tools/gpu_step.sh 300 $out/ab_shard8.log env WLD_AB_SHARD=8 python3 tools/ab_builds.py --config c4 --reps 20 --rounds 3 \
  base=weightedld_amd/libweightedld.so ring3=build/exp/ring3/libweightedld.so || exit 1
echo done
