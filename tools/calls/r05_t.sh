#!/bin/bash
# round-5 GPU call T: the item kernel with lane classes two at a time (8
# independent chains per wave; four / five workgroups per CU) at C2, its wave
# timeline, C4 LD blocks (candidate launch) A/B, and the reference-order test
# suite on the four-workgroup build (bit-identical rows)
out=gpurun_out/r05t; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 400 $out/ab_c2.log python3 tools/ab_builds.py --config c2 --reps 20 --rounds 3 \
  base=weightedld_amd/libweightedld.so cp4=build/exp/i_cp4/libweightedld.so cp5=build/exp/i_cp5/libweightedld.so || exit 1
tools/gpu_step.sh 400 $out/ab_ldb.log env WLD_AB_DATA=ldblocks python3 tools/ab_builds.py --config c4 --reps 10 --rounds 2 \
  base=weightedld_amd/libweightedld.so cp4=build/exp/i_cp4/libweightedld.so || exit 1
tools/gpu_step.sh 200 $out/item_trace_cp4.log python3 tools/item_trace.py build/exp/i_cp4_trace/libweightedld.so c2 20 || exit 1
tools/gpu_step.sh 700 $out/tests_refsums_cp4.log env WLD_LIB_PATH=build/exp/i_cp4/libweightedld.so python3 -u -m pytest -x -q \
  --timeout 300 --timeout-method thread tests/test_gpu_refsums.py tests/test_gpu_parity.py -k "not full_bench and not c5_ldblocks" || exit 1
echo done
