#!/bin/bash
# round-6 GPU call Y: candidate items with two sub-blocks per wave (A operands
# formed once for both; in-tree build) against one per wave (item1): the
# candidate tests on the in-tree build first, then A/B on LD blocks
out=gpurun_out/r06y; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 600 $out/tests.log python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_refsums.py tests/test_gpu_i8pairs.py tests/test_gpu_screen.py -m gpu || exit $?
B="item1=build/exp/item1/libweightedld.so pairs=weightedld_amd/libweightedld.so"
WLD_AB_DATA=ldblocks tools/gpu_step.sh 300 $out/ab_ldb.log python tools/ab_builds.py --config c4 --reps 20 --rounds 5 $B || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_sq -o sq -- python3 bench.py --steps 5 --warmup 2 --settle-s 0 --no-cpu-baseline --data ldblocks > $out/pmc_sq.log 2>&1 || exit $?
echo done
