#!/bin/bash
# GPU test suite only (screen tests first), for iteration.
out=gpurun_out/${1:-r02t}
mkdir -p $out
export TMPDIR=/tmp
tools/gpu_step.sh 300 $out/screen_tests.txt python -u -m pytest tests/test_gpu_screen.py -v --timeout 200 --timeout-method thread || exit $?
tools/gpu_step.sh 600 $out/gpu_tests.txt python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread || exit $?
echo done
