#!/bin/bash
# round-3 GPU call AY: the shipped build after the last reverts — smoke() and
# the default bench (CPU baseline, oracle row check)
out=gpurun_out/r03ay; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 200 $out/smoke.txt python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py || exit $?
echo done
