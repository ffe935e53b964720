#!/bin/bash
# round-6 GPU call S: candidate items with their stage operands staged through
# a per-wave LDS ring by LDS-DMA (in-tree build, 4 workgroups per CU; lds5: 5)
# against HEAD's fragment-shaped global loads: A/B on LD blocks, SQ counters;
# the candidate/screen/fp6/parity tests on the in-tree build
out=gpurun_out/r06s; mkdir -p $out; export TMPDIR=/tmp
B="head=build/exp/head/libweightedld.so lds4=weightedld_amd/libweightedld.so lds5=build/exp/lds5/libweightedld.so"
WLD_AB_DATA=ldblocks tools/gpu_step.sh 300 $out/ab_ldb.log python tools/ab_builds.py --config c4 --reps 20 --rounds 4 $B || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_sq -o sq -- python3 bench.py --steps 5 --warmup 2 --settle-s 0 --no-cpu-baseline --data ldblocks > $out/pmc_sq.log 2>&1 || exit $?
tools/gpu_step.sh 900 $out/tests.log python3 -u -m pytest -x -v --durations=10 --timeout 150 --timeout-method thread tests/test_gpu_refsums.py tests/test_gpu_screen.py tests/test_gpu_i8pairs.py tests/test_gpu_fp6.py -m gpu || exit $?
echo done
