#!/bin/bash
# round-3 GPU call V: C4 threshold sweep, the default (lib.rs's order) and the
# exact mode: where the screen, the two-plane screen and the full kernels take over
out=gpurun_out/r03v; mkdir -p $out; export TMPDIR=/tmp
for t in 0.1 0.02 0.01 0.005 0.002; do
tools/gpu_step.sh 200 $out/c4_thr${t}.log python bench.py --thr $t --steps 50 --warmup 5 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/c4_thr${t}_exact.log python bench.py --thr $t --exact-sums --steps 50 --warmup 5 --no-cpu-baseline || exit $?
done
echo done
