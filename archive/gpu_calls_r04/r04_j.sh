#!/bin/bash
# round-4 GPU call J: the fp6 give-up's cost at LD blocks; the N>1 step
# path's host share (1/8, 1/16, 1/64 shard rehearsals, a cProfile of 1/64)
out=gpurun_out/r04j; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 200 $out/abandon_timing.txt python tools/fp6_abandon_timing.py || exit $?
for k in 8 16 64; do
  tools/gpu_step.sh 200 $out/shard${k}.log python bench.py --rehearse-dist --rehearse-shard $k --no-cpu-baseline || exit $?
done
tools/gpu_step.sh 200 $out/cprofile64.txt python -m cProfile -s tottime bench.py --rehearse-dist --rehearse-shard 64 --no-cpu-baseline --steps 2000 --warmup 20 || exit $?
echo done
