#!/bin/bash
# round-3 GPU call L: f32 kernel with balanced sub-block slots and the bit-row
# compaction: parity files, then the LD-block and default benches
out=${OUT:-gpurun_out/r03l}; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 900 $out/tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_refsums.py tests/test_gpu_screen.py tests/test_gpu_parity.py -k "not full" || exit $?
tools/gpu_step.sh 200 $out/bench_c4_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c4.log python bench.py --no-cpu-baseline || exit $?
echo done
