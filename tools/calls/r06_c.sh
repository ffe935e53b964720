#!/bin/bash
# round-6 GPU call C: (1) is the unscaled fp6 x fp4 MFMA (zero scale operands)
# the same sums as the unit-scaled one, and faster?  (2) fp6 screen A/B: cur
# (in-tree), unsc (unscaled MFMA), late (arguments read at the epilogue);
# (3) the new i8 tile-pair screen: its tests, then LD-block C4 with it on/off
out=gpurun_out/r06c; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 60 $out/probe.log tools/probes/fp6_unscaled_probe || exit $?
tools/gpu_step.sh 500 $out/tests_i8pairs.log python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_i8pairs.py -m gpu || exit $?
B="cur=weightedld_amd/libweightedld.so unsc=build/exp/unsc/libweightedld.so late=build/exp/late/libweightedld.so"
tools/gpu_step.sh 300 $out/ab_c4.log python tools/ab_builds.py --config c4 --reps 30 --rounds 3 $B || exit $?
WLD_AB_SHARD=8 tools/gpu_step.sh 200 $out/ab_s8.log python tools/ab_builds.py --config c4 --reps 40 --rounds 3 $B || exit $?
WLD_AB_DATA=ldblocks tools/gpu_step.sh 300 $out/ab_ldb.log python tools/ab_builds.py --config c4 --reps 20 --rounds 3 "pairs=weightedld_amd/libweightedld.so" "tile=weightedld_amd/libweightedld.so@WLD_AB_OPTS=i8_pairs=0" || exit $?
WLD_LIB_PATH=build/exp/unsc/libweightedld.so tools/gpu_step.sh 400 $out/tests_unsc.log python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fp6.py -m gpu || exit $?
echo done
