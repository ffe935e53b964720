#!/bin/bash
# round-4 GPU call U: bench tests after the N=1-only CPU baseline change; the
# rehearsed 1/8 and 1/4 shards on the end-of-round tree
out=gpurun_out/r04u; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 600 $out/tests_bench.log python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_bench.py || exit $?
tools/gpu_step.sh 200 $out/bench_shard8.log python bench.py --rehearse-dist --rehearse-shard 8 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_shard4.log python bench.py --rehearse-dist --rehearse-shard 4 --no-cpu-baseline || exit $?
echo done
