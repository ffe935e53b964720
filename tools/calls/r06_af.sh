#!/bin/bash
# round-6 GPU call AF: the row gather's copy in batches of 2 / 4 / 8 rows
# (45-99 VGPRs) against 16 (170 VGPRs: two gather waves per SIMD displace
# two of the next step's three screen waves while they run); LD blocks
# through bench.py, alternating; C2 for the batch 4 build
out=gpurun_out/r06af; mkdir -p $out; export TMPDIR=/tmp
for i in 1 2; do
  tools/gpu_step.sh 300 $out/ldb_b16_$i.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
  for b in 2 4 8; do
    WLD_LIB_PATH=build/exp/gb$b/libweightedld.so tools/gpu_step.sh 300 $out/ldb_b${b}_$i.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
  done
done
tools/gpu_step.sh 200 $out/c2_b16.log python bench.py --config c2 --no-cpu-baseline || exit $?
WLD_LIB_PATH=build/exp/gb4/libweightedld.so tools/gpu_step.sh 200 $out/c2_b4.log python bench.py --config c2 --no-cpu-baseline || exit $?
echo done
