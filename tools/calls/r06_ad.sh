#!/bin/bash
# round-6 GPU call AD: the row gather's grid 512 (in-tree) / 1,024 / 2,048
# workgroups, LD blocks through bench.py (order phase and step), alternating
out=gpurun_out/r06ad; mkdir -p $out; export TMPDIR=/tmp
for i in 1 2; do
  tools/gpu_step.sh 300 $out/ldb_g512_$i.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
  WLD_LIB_PATH=build/exp/gg1024/libweightedld.so tools/gpu_step.sh 300 $out/ldb_g1024_$i.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
  WLD_LIB_PATH=build/exp/gg2048/libweightedld.so tools/gpu_step.sh 300 $out/ldb_g2048_$i.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
done
echo done
