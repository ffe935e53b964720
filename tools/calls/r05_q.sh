#!/bin/bash
# round-5 GPU call Q: the candidate-entry guard test (WLD_OPT_TEST_GUARD) and
# the screen suite; then call P's C2 diagnostics
out=gpurun_out/r05q; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 600 $out/tests_screen.log python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_screen.py || exit 1
tools/calls/r05_p.sh
