#!/bin/bash
# round-3 GPU call B: smoke + the whole -m gpu suite
out=gpurun_out/r03b; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 120 $out/pk_probe.txt tools/probes/pk_probe || exit $?
tools/gpu_step.sh 200 $out/smoke.txt python -c "import __graft_entry__ as g; g.smoke()" || exit $?
tools/gpu_step.sh 1000 $out/gpu_tests.txt python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread || exit $?
echo done
