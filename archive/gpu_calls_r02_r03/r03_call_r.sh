#!/bin/bash
# round-3 GPU call R: lib.rs-order kernel, next-stage register prefetch A/B
# (LD-block candidates at thr 0.05, every tile at thr 0), then the parity tests
out=gpurun_out/r03r; mkdir -p $out; export TMPDIR=/tmp
WLD_AB_DATA=ldblocks timeout -k 10 400 python tools/ab_builds.py --config c4 --reps 10 --rounds 3 pf0=build/exp/pf0/libweightedld.so pf1=build/exp/pf1/libweightedld.so > $out/ab_ldb.txt 2>&1 || { echo "ab ldb failed $?"; exit 1; }
timeout -k 10 400 python tools/ab_builds.py --config c4 --thr 0 --reps 3 --rounds 2 pf0=build/exp/pf0/libweightedld.so pf1=build/exp/pf1/libweightedld.so > $out/ab_thr0.txt 2>&1 || { echo "ab thr0 failed $?"; exit 1; }
tools/gpu_step.sh 600 $out/tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_refsums.py -k "not full" || exit $?
echo done
