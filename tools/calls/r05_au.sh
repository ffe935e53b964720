#!/bin/bash
# round-5 GPU call AU: the in-tree library as rebuilt last (timing macro added,
# default path unchanged): fp6 / screen / parity tests, smoke, one C4 bench line
out=gpurun_out/r05au; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 600 $out/tests.log python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_fp6.py tests/test_gpu_screen.py tests/test_gpu_parity.py -m gpu || exit 1
tools/gpu_step.sh 120 $out/smoke.txt python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
tools/gpu_step.sh 200 $out/bench_c4.log python bench.py || exit $?
echo done
