#!/bin/bash
# round-4 GPU call A: the new tests first (launcher at --gpus 2 over gloo,
# pre-pass vs oracle, C5 rows, CLI progress bars), then the whole -m gpu suite,
# smoke(), the default bench and C2 / LD-block lines
out=gpurun_out/r04a; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 600 $out/new_tests.txt python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_bench.py tests/test_gpu_prepass.py tests/test_gpu_parity.py::test_cli_progress_bars \
  "tests/test_gpu_refsums.py::test_c5_ldblocks_rows_bit_exact" "tests/test_gpu_refsums.py::test_report_full_bench_workloads" || exit $?
tools/gpu_step.sh 900 $out/gpu_tests.txt python -u -m pytest tests -m gpu -q -rf --timeout 400 --timeout-method thread \
  --deselect tests/test_bench.py --deselect tests/test_gpu_prepass.py --deselect tests/test_gpu_refsums.py::test_c5_ldblocks_rows_bit_exact --deselect tests/test_gpu_refsums.py::test_report_full_bench_workloads || exit $?
tools/gpu_step.sh 200 $out/smoke.txt python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py || exit $?
tools/gpu_step.sh 200 $out/bench_c2.log python bench.py --config c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
echo done
