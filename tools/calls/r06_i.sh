#!/bin/bash
# round-6 GPU call I: the N=1 step loop's serialization (WLD_PIPE_SERIALIZE
# pair, the default, against 0: screens free to overlap) over C4, LD blocks
# and C2, interleaved, 3 reps; the read-first build (next stage's copies
# issued after this stage's A reads) against the tree's build through bench.py
# at C4 and rank 0's 1/8 shard
out=gpurun_out/r06i; mkdir -p $out; export TMPDIR=/tmp
RF=build/exp/readfirst/libweightedld.so
for i in 1 2 3; do
  for m in pair 0; do
    WLD_PIPE_SERIALIZE=$m tools/gpu_step.sh 200 $out/c4_${m}_$i.log python bench.py --no-cpu-baseline || exit $?
    WLD_PIPE_SERIALIZE=$m tools/gpu_step.sh 200 $out/ldb_${m}_$i.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
    WLD_PIPE_SERIALIZE=$m tools/gpu_step.sh 200 $out/c2_${m}_$i.log python bench.py --config c2 --no-cpu-baseline || exit $?
  done
  WLD_LIB_PATH=$RF tools/gpu_step.sh 200 $out/c4_rf_$i.log python bench.py --no-cpu-baseline || exit $?
  tools/gpu_step.sh 200 $out/s8_cur_$i.log python bench.py --rehearse-dist --rehearse-shard 8 --no-cpu-baseline || exit $?
  WLD_LIB_PATH=$RF tools/gpu_step.sh 200 $out/s8_rf_$i.log python bench.py --rehearse-dist --rehearse-shard 8 --no-cpu-baseline || exit $?
done
echo done
