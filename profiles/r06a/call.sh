#!/bin/bash
# round-6 GPU call A: pruned kernels (no experiment switches), planted-LD
# full-size fp6 tests, ADVICE r5 fixes, 8-rank launcher: the whole GPU suite,
# smoke, one default bench line (with the planted rows check)
out=gpurun_out/r06a; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 1000 $out/tests.log python3 -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests -m gpu || exit 1
tools/gpu_step.sh 120 $out/smoke.txt python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py || exit $?
echo done
