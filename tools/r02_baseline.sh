#!/bin/bash
# Round-2 baseline on a fresh box: GPU tests, C4 bench, non-pipelined rocprof stats.
out=gpurun_out/r02a
mkdir -p $out
export TMPDIR=/tmp
tools/gpu_step.sh 400 $out/gpu_tests.txt python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o c4 -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pipeline > $out/prof.log 2>&1 || { echo "rocprof failed $?"; exit 1; }
echo done
