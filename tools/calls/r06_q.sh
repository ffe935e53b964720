#!/bin/bash
# round-6 GPU call Q: candidate items in buckets by the screen workgroup's
# XCD queue, each XCD's workgroups taking their own bucket first (in-tree
# build) against HEAD's one list dealt over the CUs: A/B on LD blocks; L2
# and SQ counters of both on LD blocks; the candidate/screen/fp6 tests
out=gpurun_out/r06q; mkdir -p $out; export TMPDIR=/tmp
B="head=build/exp/head/libweightedld.so xcd=weightedld_amd/libweightedld.so"
WLD_AB_DATA=ldblocks tools/gpu_step.sh 300 $out/ab_ldb.log python tools/ab_builds.py --config c4 --reps 20 --rounds 4 $B || exit $?
for v in head xcd; do
  lib=build/exp/head/libweightedld.so; [ $v = xcd ] && lib=weightedld_amd/libweightedld.so
  WLD_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_l2_$v -o l2 -- python3 bench.py --steps 5 --warmup 2 --settle-s 0 --no-cpu-baseline --data ldblocks > $out/pmc_l2_$v.log 2>&1 || exit $?
  WLD_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_sq_$v -o sq -- python3 bench.py --steps 5 --warmup 2 --settle-s 0 --no-cpu-baseline --data ldblocks > $out/pmc_sq_$v.log 2>&1 || exit $?
done
tools/gpu_step.sh 900 $out/tests.log python3 -u -m pytest -x -v --durations=10 --timeout 150 --timeout-method thread tests/test_gpu_refsums.py tests/test_gpu_screen.py tests/test_gpu_i8pairs.py tests/test_gpu_fp6.py -m gpu || exit $?
echo done
