#!/bin/bash
# round-6 GPU call W: the i8 tile-pair screen with a three-buffer LDS-DMA ring
# (copies two stages ahead, counted vmcnt, raw barrier; 48 KB, still three
# workgroups per CU) against two buffers: A/B on LD blocks; the i8/screen
# tests on it
out=gpurun_out/r06w; mkdir -p $out; export TMPDIR=/tmp
B="base=weightedld_amd/libweightedld.so i8r3=build/exp/i8r3/libweightedld.so"
WLD_AB_DATA=ldblocks tools/gpu_step.sh 300 $out/ab_ldb.log python tools/ab_builds.py --config c4 --reps 20 --rounds 5 $B || exit $?
WLD_LIB_PATH=build/exp/i8r3/libweightedld.so tools/gpu_step.sh 600 $out/tests_i8r3.log python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_i8pairs.py tests/test_gpu_screen.py -m gpu || exit $?
echo done
