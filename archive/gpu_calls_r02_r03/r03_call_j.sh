#!/bin/bash
# round-3 GPU call J: repeat the depth-3 unserialized pipeline against depth-2
# "pair" on 1/8, 1/4, 1/2 shards and the whole C4 (variance check)
out=gpurun_out/r03j; mkdir -p $out; export TMPDIR=/tmp
for rep in 1 2 3; do for sh in 8 4 2 1; do
WLD_PIPE_SERIALIZE=0 tools/gpu_step.sh 200 $out/s${sh}_d3_0_r$rep.log python bench.py --rehearse-dist --rehearse-shard $sh --pipe-depth 3 --no-cpu-baseline || exit $?
WLD_PIPE_SERIALIZE=pair tools/gpu_step.sh 200 $out/s${sh}_d2_pair_r$rep.log python bench.py --rehearse-dist --rehearse-shard $sh --pipe-depth 2 --no-cpu-baseline || exit $?
done; done
echo done
