#!/bin/bash
# Round-2 iteration: GPU tests (screen/prefilter first), C4 bench screened and unscreened.
out=gpurun_out/${1:-r02b}
mkdir -p $out
export TMPDIR=/tmp
tools/gpu_step.sh 300 $out/screen_tests.txt python -u -m pytest tests/test_gpu_screen.py -x -v --timeout 200 --timeout-method thread || exit $?
tools/gpu_step.sh 500 $out/gpu_tests.txt python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit $?
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $out/bench_c4_noscreen.log python bench.py --no-cpu-baseline --no-screen || exit $?
tools/gpu_step.sh 300 $out/bench_c5.log python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline || exit $?
echo done
