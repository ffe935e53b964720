#!/bin/bash
# Quick GPU iteration: screen tests, C4/C5 bench lines, optional A/B of builds.  -> gpurun_out/TAG/
tag=${1:-r02q}; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
tools/gpu_step.sh 300 $out/screen_tests.txt python -u -m pytest tests/test_gpu_screen.py -q -x --timeout 300 --timeout-method thread || exit $?
tools/gpu_step.sh 200 $out/bench_c4.log python bench.py --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $out/bench_c5.log python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline || exit $?
if [ $# -gt 0 ]; then
  tools/gpu_step.sh 400 $out/ab.txt python tools/ab_builds.py --config c4 --reps 20 --rounds 3 "$@" || exit $?
fi
echo done
