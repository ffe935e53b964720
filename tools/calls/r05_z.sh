#!/bin/bash
# round-5 GPU call Z: first-pass timings after moving the per-data-set builds
# to load, the fp6/screen/parity tests, and the headline line
out=gpurun_out/r05z; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 200 $out/first_rand.log python3 tools/first_pass.py random 0.05 || exit $?
tools/gpu_step.sh 200 $out/first_ldb.log python3 tools/first_pass.py ldblocks 0.05 || exit $?
tools/gpu_step.sh 700 $out/tests.log python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_fp6.py tests/test_gpu_parity.py tests/test_gpu_multi.py -k "not full_size" || exit $?
tools/gpu_step.sh 200 $out/bench_c4.log python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
echo done
