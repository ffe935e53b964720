#!/bin/bash
# round-5 GPU call AD: the item kernel with each stage's A operands formed once
# per workgroup and shared through LDS (six / seven workgroups per CU) at C2;
# the reference-order suite on it (bit-identical rows)
out=gpurun_out/r05ad; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 400 $out/ab_c2.log python3 tools/ab_builds.py --config c2 --reps 20 --rounds 3 \
  base=weightedld_amd/libweightedld.so ash6=build/exp/i_ash/libweightedld.so ash7=build/exp/i_ash7/libweightedld.so || exit 1
tools/gpu_step.sh 700 $out/tests_ash.log env WLD_LIB_PATH=build/exp/i_ash/libweightedld.so python3 -u -m pytest -x -q \
  --timeout 300 --timeout-method thread tests/test_gpu_refsums.py tests/test_gpu_parity.py tests/test_gpu_screen.py -k "not full_bench and not c5_ldblocks" || exit 1
echo done
