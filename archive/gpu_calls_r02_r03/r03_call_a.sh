#!/bin/bash
# round-3 GPU call A: new GPU tests (ref sums, progress, screen, parity) and the packed-f32 probe
out=gpurun_out/r03a; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 420 $out/pk_hazard.txt python -u tools/probes/pk_hazard.py --reps 2 || exit $?
tools/gpu_step.sh 900 $out/gpu_tests.txt python -u -m pytest tests/test_gpu_refsums.py tests/test_gpu_parity.py tests/test_gpu_screen.py -m gpu -v -rf --timeout 300 --timeout-method thread || exit $?
echo done
