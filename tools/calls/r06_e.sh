#!/bin/bash
# round-6 GPU call E: persistent tile-pair fp6 screen (WLD_F6_PERSIST) A/B at
# C4, C5 and the 1/8 shard, and its fp6/screen tests; the N>1 step path with
# the row counts through host shared memory (HostCountExchange) against the
# RCCL count all_gather (rehearsed 1/8 shard), and its GPU tests
out=gpurun_out/r06e; mkdir -p $out; export TMPDIR=/tmp
B="cur=weightedld_amd/libweightedld.so persist=build/exp/persist/libweightedld.so"
tools/gpu_step.sh 300 $out/ab_c4.log python tools/ab_builds.py --config c4 --reps 30 --rounds 3 $B || exit $?
tools/gpu_step.sh 300 $out/ab_c5.log python tools/ab_builds.py --config c5 --reps 6 --rounds 2 $B || exit $?
WLD_AB_SHARD=8 tools/gpu_step.sh 200 $out/ab_s8.log python tools/ab_builds.py --config c4 --reps 40 --rounds 3 $B || exit $?
for i in 1 2; do
tools/gpu_step.sh 200 $out/shard8_shm_$i.log python bench.py --rehearse-dist --rehearse-shard 8 --no-cpu-baseline --counts shm || exit $?
tools/gpu_step.sh 200 $out/shard8_coll_$i.log python bench.py --rehearse-dist --rehearse-shard 8 --no-cpu-baseline --counts collective || exit $?
done
tools/gpu_step.sh 600 $out/tests_dist.log python3 -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_gpu_dist.py tests/test_bench.py -m gpu || exit $?
WLD_LIB_PATH=build/exp/persist/libweightedld.so tools/gpu_step.sh 400 $out/tests_persist.log python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fp6.py tests/test_gpu_screen.py -m gpu || exit $?
echo done
