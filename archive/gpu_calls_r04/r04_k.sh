#!/bin/bash
# round-4 GPU call K: the fp6 give-up without repeated marks: fp6 tests, the
# give-up's cost at LD blocks, the LD-block bench line
out=gpurun_out/r04k; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 400 $out/fp6_tests.txt python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fp6.py || exit $?
tools/gpu_step.sh 200 $out/abandon_timing.txt python tools/fp6_abandon_timing.py || exit $?
tools/gpu_step.sh 200 $out/bench_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
for d in 3 4 6; do
  tools/gpu_step.sh 200 $out/shard8_depth$d.log python bench.py --rehearse-dist --rehearse-shard 8 --pipe-depth $d --no-cpu-baseline || exit $?
done
echo done
