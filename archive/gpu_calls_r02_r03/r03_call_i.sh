#!/bin/bash
# round-3 GPU call I: pipeline depth x device serialization A/B (rehearsed
# N>1 loop) on rank 0's 1/8 and 1/4 shards and the whole C4
out=gpurun_out/r03i; mkdir -p $out; export TMPDIR=/tmp
for sh in 8 4 1; do for d in 2 3; do for s in pair 0; do
WLD_PIPE_SERIALIZE=$s tools/gpu_step.sh 200 $out/s${sh}_d${d}_$s.log python bench.py --rehearse-dist --rehearse-shard $sh --pipe-depth $d --no-cpu-baseline || exit $?
done; done; done
echo done
