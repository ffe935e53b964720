#!/bin/bash
# round-4 GPU call D: the fp6 x fp4 MFMA probe, then the fp6 screen and the
# LDS-free reference-order item kernel — targeted tests, A/B against the
# round-3 shape and the i8 screen, bench lines
out=gpurun_out/r04d; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 60 $out/fp6_probe.txt tools/probes/fp6_probe || exit $?
tools/gpu_step.sh 900 $out/new_tests.txt python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_fp6.py tests/test_gpu_parity.py::test_progress_once_per_chunk_screened \
  tests/test_gpu_parity.py::test_progress_once_per_chunk_config2 tests/test_gpu_parity.py::test_contexts_on_one_stream \
  tests/test_gpu_refsums.py tests/test_gpu_screen.py || exit $?
tools/gpu_step.sh 300 $out/ab_c2.txt python tools/ab_builds.py --config c2 --thr 0.0 --reps 20 --rounds 3 \
  items=weightedld_amd/libweightedld.so r3=build/exp/r3items/libweightedld.so || exit $?
WLD_AB_DATA=ldblocks tools/gpu_step.sh 300 $out/ab_ldb.txt python tools/ab_builds.py --config c4 --reps 10 --rounds 3 \
  items=weightedld_amd/libweightedld.so r3=build/exp/r3items/libweightedld.so || exit $?
tools/gpu_step.sh 300 $out/ab_c4_fp6.txt python tools/ab_builds.py --config c4 --reps 20 --rounds 3 \
  fp6=weightedld_amd/libweightedld.so@WLD_AB_OPTS=screen_fp6=2 i8=weightedld_amd/libweightedld.so@WLD_AB_OPTS=screen_fp6=0 || exit $?
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py || exit $?
tools/gpu_step.sh 200 $out/bench_c2.log python bench.py --config c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $out/bench_c5.log python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline || exit $?
echo done
