#!/bin/bash
# round-3 GPU call AO: pipeline depth sweep of the rehearsed N>1 step (rank 0's
# 1/2, 1/4, 1/8, 1/16 shards of C4), two passes interleaved
out=gpurun_out/r03ao; mkdir -p $out; export TMPDIR=/tmp
for pass in 1 2; do for s in 8 16 4 2; do for d in 3 4 6 8; do
tools/gpu_step.sh 200 $out/p${pass}_shard${s}_d${d}.log python bench.py --no-cpu-baseline --rehearse-dist --rehearse-shard $s --pipe-depth $d --steps 400 --warmup 40 || exit $?
done; done; done
echo done
