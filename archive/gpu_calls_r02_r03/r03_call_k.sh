#!/bin/bash
# round-3 GPU call K: reference-order kernel with transposed 16-groups (dword
# LDS reads, per-sub-block MFMA skipping): bit-exact tests, then the LD-block
# and default benches
out=gpurun_out/r03k; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 600 $out/tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_refsums.py tests/test_gpu_screen.py -k "not full" || exit $?
tools/gpu_step.sh 200 $out/bench_c4_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c4.log python bench.py --no-cpu-baseline || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o ldb -- \
  python3 bench.py --data ldblocks --steps 30 --warmup 5 --no-cpu-baseline > $out/prof_ldb.log 2>&1 || { echo "rocprof failed $?"; exit 1; }
echo done
