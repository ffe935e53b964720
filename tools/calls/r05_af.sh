#!/bin/bash
# round-5 GPU call AF: the reference-order / parity / screen / fp6 suites on the
# default build (A operands shared in full runs only), C2 and LD-block lines
out=gpurun_out/r05af; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 900 $out/tests.log python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_refsums.py tests/test_gpu_parity.py tests/test_gpu_screen.py tests/test_gpu_fp6.py -k "not full_bench and not c5_ldblocks" || exit 1
tools/gpu_step.sh 200 $out/bench_c2.log python bench.py --config c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
echo done
