#!/bin/bash
# round-6 GPU call AL: the candidate item launch's grid (512 / 768 / 1,024
# workgroups) in the pipelined LD-block step, where it runs beside the next
# pass's screen (the A/B harness runs one pass at a time), bench.py, alternating
out=gpurun_out/r06al; mkdir -p $out; export TMPDIR=/tmp
for i in 1 2; do
  tools/gpu_step.sh 300 $out/ldb_g1024_$i.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
  for g in 512 768; do
    WLD_LIB_PATH=build/exp/ig$g/libweightedld.so tools/gpu_step.sh 300 $out/ldb_g${g}_$i.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
  done
done
echo done
