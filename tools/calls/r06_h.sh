#!/bin/bash
# round-6 GPU call H: the next stage's copies issued after this stage's A
# reads (A/B); the N=1 step loop's serialization at C4 (pair kernels
# queued behind each other, the default, against screens free to overlap);
# then the final tree's lines: C4 (200/20 and the driver's 20/5), LD blocks,
# C2, C5, rank 0's 1/8 and 1/4 shards through the N>1 path, the first pass of
# a fresh context; the rocprofv3 kernel statistics of the headline command
out=gpurun_out/r06h; mkdir -p $out; export TMPDIR=/tmp
B="cur=weightedld_amd/libweightedld.so readfirst=build/exp/readfirst/libweightedld.so"
tools/gpu_step.sh 300 $out/ab_c4.log python tools/ab_builds.py --config c4 --reps 30 --rounds 3 $B || exit $?
WLD_AB_SHARD=8 tools/gpu_step.sh 200 $out/ab_s8.log python tools/ab_builds.py --config c4 --reps 40 --rounds 3 $B || exit $?
for i in 1 2; do
  tools/gpu_step.sh 200 $out/c4_pair_$i.log python bench.py --no-cpu-baseline || exit $?
  WLD_PIPE_SERIALIZE=0 tools/gpu_step.sh 200 $out/c4_free_$i.log python bench.py --no-cpu-baseline || exit $?
  WLD_PIPE_SERIALIZE=0 tools/gpu_step.sh 200 $out/c4_free3_$i.log python bench.py --no-cpu-baseline --pipe-depth 3 || exit $?
done
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py || exit $?
tools/gpu_step.sh 200 $out/bench_c4_20_5.log python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $out/bench_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $out/bench_c2.log python bench.py --config c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 400 $out/bench_c5.log python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/shard8.log python bench.py --rehearse-dist --rehearse-shard 8 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/shard4.log python bench.py --rehearse-dist --rehearse-shard 4 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/first_random.log python tools/first_pass.py random || exit $?
tools/gpu_step.sh 200 $out/first_ldb.log python tools/first_pass.py ldblocks || exit $?
tools/gpu_step.sh 300 $out/prof_c4.log rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c4 -o c4 -- python3 bench.py --no-cpu-baseline || exit $?
echo done
