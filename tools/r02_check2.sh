#!/bin/bash
# GPU tests (new files first) + C4 benches: default, unscreened, 4-plane (wide weights) screened/unscreened, C2.
out=gpurun_out/${1:-r02e}
mkdir -p $out
export TMPDIR=/tmp
tools/gpu_step.sh 400 $out/screen_tests.txt python -u -m pytest tests/test_gpu_screen.py -v -s --timeout 200 --timeout-method thread || exit $?
tools/gpu_step.sh 200 $out/bench_c4.log python bench.py --no-cpu-baseline --steps 100 || exit $?
tools/gpu_step.sh 200 $out/bench_c4_wide.log python bench.py --no-cpu-baseline --wide-weights --steps 50 || exit $?
tools/gpu_step.sh 200 $out/bench_c4_wide_noscreen.log python bench.py --no-cpu-baseline --wide-weights --no-screen --steps 20 || exit $?
tools/gpu_step.sh 200 $out/bench_c2.log python bench.py --no-cpu-baseline --config c2 || exit $?
tools/gpu_step.sh 600 $out/gpu_tests.txt python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread || exit $?
echo done
