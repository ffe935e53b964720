#!/bin/bash
# round-3 GPU call AA: the other BASELINE configs in the default mode (C2 thr 0:
# every pair; C5 thr 0.05) and C2 in the exact mode
out=gpurun_out/r03aa; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 300 $out/c2.log python bench.py --config c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $out/c2_exact.log python bench.py --config c2 --exact-sums --no-cpu-baseline || exit $?
tools/gpu_step.sh 400 $out/c5.log python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline || exit $?
echo done
