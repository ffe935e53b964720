#!/bin/bash
# round-4 GPU call I: the N>1 step path's host share at small shards
# (rehearsal through an RCCL group of one): 1/8, 1/16, 1/64 shards with the
# pinned count copy and with the synchronous count read; a cProfile of the
# 1/64 rehearsal; the dist GPU tests
out=gpurun_out/r04i; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 400 $out/gpu_dist_tests.txt python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_dist.py tests/test_bench.py || exit $?
for k in 8 16 64; do
  tools/gpu_step.sh 200 $out/shard${k}_pinned.log python bench.py --rehearse-dist --rehearse-shard $k --no-cpu-baseline || exit $?
  WLD_DIST_PINNED=0 tools/gpu_step.sh 200 $out/shard${k}_sync.log python bench.py --rehearse-dist --rehearse-shard $k --no-cpu-baseline || exit $?
done
tools/gpu_step.sh 200 $out/shard8_pinned_b.log python bench.py --rehearse-dist --rehearse-shard 8 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/cprofile64.txt python -m cProfile -s tottime bench.py --rehearse-dist --rehearse-shard 64 --no-cpu-baseline --steps 2000 --warmup 20 || exit $?
echo done
