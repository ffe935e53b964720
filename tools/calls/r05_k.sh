#!/bin/bash
# round-5 GPU call K: fp6 sample run (tests, first pass vs steady on linkage
# blocks and random data), capped-grid gather (parity tests with rows), LD-block bench
out=gpurun_out/r05k; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 500 $out/tests.log python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_fp6.py tests/test_gpu_parity.py -k "not full_size" || exit 1
tools/gpu_step.sh 200 $out/first_ldb.log python3 tools/first_pass.py ldblocks 0.05 || exit 1
tools/gpu_step.sh 200 $out/first_rand.log python3 tools/first_pass.py random 0.05 || exit 1
tools/gpu_step.sh 300 $out/bench_ldb.log python3 bench.py --data ldblocks --steps 50 --warmup 10 --no-cpu-baseline || exit 1
tools/gpu_step.sh 300 $out/bench_c2.log python3 bench.py --config c2 --steps 200 --warmup 20 --no-cpu-baseline || exit 1
echo done
