#!/bin/bash
# round-3 GPU call W: exact candidate pairs + per-pair lib.rs sums (screened 4):
# bit-exact tests, then the C4 threshold sweep in the default mode
out=${OUT:-gpurun_out/r03w}; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 600 $out/tests.log python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_refsums.py -k "policy or ref_pairs" || exit $?
for t in 0.01 0.005 0.002; do
tools/gpu_step.sh 200 $out/c4_thr${t}.log python bench.py --thr $t --steps 50 --warmup 5 --no-cpu-baseline || exit $?
done
echo done
