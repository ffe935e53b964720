#!/bin/bash
# round-6 GPU call AA: a persistent fp6 screen (three resident workgroups per
# CU drain their XCD's entry queue from a per-queue counter; the next entry
# fetched during the second-last stage and its first stage copied during the
# epilogue, behind raw barriers) against the per-entry launch: fp6 tests on
# it first, then A/B at C4, the 1/8 shard, C5
out=gpurun_out/r06aa; mkdir -p $out; export TMPDIR=/tmp
WLD_LIB_PATH=build/exp/persist/libweightedld.so tools/gpu_step.sh 400 $out/tests_fp6.log python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_fp6.py -m gpu || exit $?
B="base=weightedld_amd/libweightedld.so persist=build/exp/persist/libweightedld.so"
tools/gpu_step.sh 300 $out/ab_c4.log python tools/ab_builds.py --config c4 --reps 30 --rounds 4 $B || exit $?
WLD_AB_SHARD=8 tools/gpu_step.sh 300 $out/ab_s8.log python tools/ab_builds.py --config c4 --reps 40 --rounds 3 $B || exit $?
tools/gpu_step.sh 300 $out/ab_c5.log python tools/ab_builds.py --config c5 --reps 6 --rounds 2 $B || exit $?
echo done
