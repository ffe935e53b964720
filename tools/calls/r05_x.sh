#!/bin/bash
# round-5 GPU call X: rehearsed shards through the N>1 step path with the fp6
# screen on single tiles (default below 16,384 tiles) vs tile pairs, interleaved
out=gpurun_out/r05x; mkdir -p $out; export TMPDIR=/tmp
for rep in 1 2; do
  for k in 8 4; do
    tools/gpu_step.sh 200 $out/shard${k}_single_$rep.log python bench.py --rehearse-dist --rehearse-shard $k --no-cpu-baseline || exit $?
    tools/gpu_step.sh 200 $out/shard${k}_pairs_$rep.log env WLD_BENCH_OPTS="fp6_pairs_min_tiles=0" python bench.py \
      --rehearse-dist --rehearse-shard $k --no-cpu-baseline || exit $?
  done
done
echo done
