#!/bin/bash
# round-4 GPU call L (tree at the end of the round): the whole -m gpu suite,
# smoke(), the headline bench line
out=gpurun_out/r04l; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 1000 $out/gpu_tests.txt python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests || exit $?
tools/gpu_step.sh 120 $out/smoke.txt python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py || exit $?
echo done
