#!/bin/bash
# round-5 GPU call J: fp6 screen variants at C5 and on C4-size linkage blocks
# (forced fp6 there), one-at-a-time harness; then the N>1 step path with the
# torch-owned step streams and the pinned count read: GPU dist tests and the
# 1/8-shard rehearsal (must exit 0)
out=gpurun_out/r05j; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 500 $out/ab_c5.log python3 tools/ab_builds.py --config c5 --reps 5 --rounds 2 \
  old=build/exp/old/libweightedld.so pairs_b4=weightedld_amd/libweightedld.so single_b4=build/exp/single_b4/libweightedld.so || exit 1
WLD_AB_DATA=ldblocks tools/gpu_step.sh 500 $out/ab_ldb.log python3 tools/ab_builds.py --config c4 --reps 5 --rounds 2 \
  old=build/exp/old/libweightedld.so@WLD_AB_OPTS=screen_fp6=2 pairs_b4=weightedld_amd/libweightedld.so@WLD_AB_OPTS=screen_fp6=2 \
  single_b4=build/exp/single_b4/libweightedld.so@WLD_AB_OPTS=screen_fp6=2 || exit 1
tools/gpu_step.sh 400 $out/tests_dist.log python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_dist.py tests/test_bench.py -m gpu || exit 1
tools/gpu_step.sh 300 $out/shard8.log python3 bench.py --rehearse-dist --rehearse-shard 8 --steps 200 --warmup 20 --no-cpu-baseline || exit 1
echo done
