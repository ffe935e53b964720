#!/bin/bash
# Tile launch order (XCD-aware vs plain rows) for the rehearsed per-rank step
# (rank 0's 1/8 and 1/4 shard of C4) and the whole C4.  -> gpurun_out/TAG/
out=gpurun_out/${1:-r02oa}; mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
for sh in 8 4 0; do
  tools/gpu_step.sh 200 $out/xcd_s${sh}_$rep.log python bench.py --rehearse-dist --rehearse-shard $sh --no-cpu-baseline || exit $?
  tools/gpu_step.sh 200 $out/rows_s${sh}_$rep.log python bench.py --rehearse-dist --rehearse-shard $sh --tile-rows --no-cpu-baseline || exit $?
done
done
echo done
