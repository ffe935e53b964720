#!/bin/bash
# round-5 GPU call AE: A operands shared through LDS in the candidate items too
# (LD blocks; C4 thr 0.01 with many candidates), and at five workgroups per CU;
# the reference-order / screen / fp6 suites on the new default
out=gpurun_out/r05ae; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 400 $out/ab_ldb.log env WLD_AB_DATA=ldblocks python3 tools/ab_builds.py --config c4 --reps 10 --rounds 3 \
  noshare=build/exp/ash0/libweightedld.so share=weightedld_amd/libweightedld.so share5=build/exp/loop5/libweightedld.so || exit 1
tools/gpu_step.sh 400 $out/ab_c4_thr02.log python3 tools/ab_builds.py --config c4 --thr 0.02 --reps 5 --rounds 2 \
  noshare=build/exp/ash0/libweightedld.so share=weightedld_amd/libweightedld.so share5=build/exp/loop5/libweightedld.so || exit 1
tools/gpu_step.sh 400 $out/ab_c2.log python3 tools/ab_builds.py --config c2 --reps 20 --rounds 2 \
  noshare=build/exp/ash0/libweightedld.so share=weightedld_amd/libweightedld.so || exit 1
tools/gpu_step.sh 900 $out/tests.log python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_refsums.py tests/test_gpu_parity.py tests/test_gpu_screen.py tests/test_gpu_fp6.py -k "not full_bench and not c5_ldblocks" || exit 1
echo done
