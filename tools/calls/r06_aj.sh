#!/bin/bash
# round-6 GPU call AJ: full runs (C2) with each wave's B rows staged through a
# two-slot LDS ring by LDS-DMA (the A-share path kept) against fragment-shaped
# B loads: parity/screen tests on it, A/B at C2, bench.py C2 both ways
out=gpurun_out/r06aj; mkdir -p $out; export TMPDIR=/tmp
WLD_LIB_PATH=build/exp/bst/libweightedld.so tools/gpu_step.sh 900 $out/tests.log python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_screen.py tests/test_gpu_parity.py -m gpu || exit $?
B="base=weightedld_amd/libweightedld.so bst=build/exp/bst/libweightedld.so"
tools/gpu_step.sh 300 $out/ab_c2.log python tools/ab_builds.py --config c2 --reps 40 --rounds 5 $B || exit $?
for i in 1 2; do
  tools/gpu_step.sh 200 $out/c2_base_$i.log python bench.py --config c2 --no-cpu-baseline || exit $?
  WLD_LIB_PATH=build/exp/bst/libweightedld.so tools/gpu_step.sh 200 $out/c2_bst_$i.log python bench.py --config c2 --no-cpu-baseline || exit $?
done
echo done
