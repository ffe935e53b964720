#!/bin/bash
# The -m gpu suite (or the given test files) on the GPU box, one call.
#   tools/calls/r03_tests.sh TAG [pytest args...]   -> gpurun_out/TAG/gpu_tests.txt
tag=${1:-r03t}; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
args=${@:-tests}
timeout -k 10 1000 python -u -m pytest $args -m gpu -v -rf --timeout 300 --timeout-method thread > $out/gpu_tests.txt 2>&1
rc=$?
tail -n 40 $out/gpu_tests.txt
exit $rc
