#!/bin/bash
out=gpurun_out/${1:-r02g}
mkdir -p $out
export TMPDIR=/tmp
tools/gpu_step.sh 250 $out/four_plane_repeat.txt python -u tools/debug/four_plane_debug2.py || exit $?
tools/gpu_step.sh 400 $out/screen_tests.txt python -u -m pytest tests/test_gpu_screen.py -v -s --timeout 300 --timeout-method thread || exit $?
tools/gpu_step.sh 200 $out/bench_c4_wide.log python bench.py --no-cpu-baseline --wide-weights --steps 50 || exit $?
tools/gpu_step.sh 200 $out/bench_c4_wide_noscreen.log python bench.py --no-cpu-baseline --wide-weights --no-screen --steps 20 || exit $?
tools/gpu_step.sh 600 $out/gpu_tests.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread || exit $?
echo done
