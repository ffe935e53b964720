#!/bin/bash
# round-6 GPU call AI (diagnostic): LD blocks with one context (steps back to
# back, every step on the same operand images) against the default two
# contexts (their images alternate in the Infinity Cache); C4 the same
out=gpurun_out/r06ai; mkdir -p $out; export TMPDIR=/tmp
for i in 1 2; do
  tools/gpu_step.sh 300 $out/ldb_two_$i.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
  tools/gpu_step.sh 300 $out/ldb_one_$i.log python bench.py --data ldblocks --no-cpu-baseline --no-pipeline || exit $?
done
tools/gpu_step.sh 300 $out/c4_one.log python bench.py --no-cpu-baseline --no-pipeline || exit $?
tools/gpu_step.sh 300 $out/c4_two.log python bench.py --no-cpu-baseline || exit $?
echo done
