#!/bin/bash
# round-4 GPU call G (final tree): the whole -m gpu suite, smoke(), the
# 2-rank launcher with per-step oracle checks
out=gpurun_out/r04_final; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 1000 $out/gpu_tests.txt python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests || exit $?
tools/gpu_step.sh 120 $out/smoke.txt python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
echo done
