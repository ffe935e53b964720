#!/bin/bash
# round-3 GPU call AB: lib.rs-order f32 kernel, operands staged through LDS vs
# straight from memory per wave (3 or 4 workgroups per CU): LD-block
# candidates, every tile of C4 at thr 0, C2 at thr 0; then the bit-exact tests
out=gpurun_out/r03ab; mkdir -p $out; export TMPDIR=/tmp
B="lds=build/exp/lds/libweightedld.so direct=build/exp/direct/libweightedld.so direct4=build/exp/direct4/libweightedld.so"
WLD_AB_DATA=ldblocks timeout -k 10 400 python tools/ab_builds.py --config c4 --reps 10 --rounds 2 $B > $out/ab_ldb.txt 2>&1 || { echo "ab ldb failed"; exit 1; }
timeout -k 10 400 python tools/ab_builds.py --config c4 --thr 0 --reps 3 --rounds 1 $B > $out/ab_c4_thr0.txt 2>&1 || { echo "ab thr0 failed"; exit 1; }
timeout -k 10 300 python tools/ab_builds.py --config c2 --reps 10 --rounds 2 $B > $out/ab_c2.txt 2>&1 || { echo "ab c2 failed"; exit 1; }
tools/gpu_step.sh 600 $out/tests.log python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_refsums.py -k "not full" || exit $?
echo done
