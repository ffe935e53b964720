#!/bin/bash
# round-3 GPU call AN: is the rehearsed N>1 step host-bound? rank 0's 1/8 and
# 1/16 shards of C4 at pipeline depth 3 (default) and 4
out=gpurun_out/r03an; mkdir -p $out; export TMPDIR=/tmp
for s in 8 16; do for d in 3 4; do
tools/gpu_step.sh 200 $out/shard${s}_d${d}.log python bench.py --no-cpu-baseline --rehearse-dist --rehearse-shard $s --pipe-depth $d --steps 400 --warmup 40 || exit $?
done; done
echo done
