#!/bin/bash
# round-4 GPU call B: the candidate-item / gather / progress-bar changes —
# targeted tests first, then the whole suite, smoke, bench lines
out=gpurun_out/r04b; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 900 $out/new_tests.txt python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py::test_cli_progress_bars tests/test_gpu_parity.py::test_progress_once_per_chunk_screened \
  tests/test_gpu_parity.py::test_progress_once_per_chunk_config2 tests/test_gpu_refsums.py tests/test_gpu_screen.py || exit $?
tools/gpu_step.sh 200 $out/bench_c2.log python bench.py --config c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py --no-cpu-baseline || exit $?
tools/gpu_step.sh 900 $out/gpu_tests.txt python -u -m pytest tests -m gpu -q -rf --timeout 400 --timeout-method thread \
  --deselect tests/test_gpu_refsums.py --deselect tests/test_gpu_screen.py || exit $?
echo done
