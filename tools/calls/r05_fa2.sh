#!/bin/bash
# round-5 final call A (wide-wave screen tree): the whole -m gpu suite and smoke()
out=gpurun_out/r05_final2; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 1100 $out/gpu_tests.txt python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests || exit $?
tools/gpu_step.sh 120 $out/smoke.txt python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
echo done
