#!/bin/bash
# round-6 GPU call R (final tree's lines; product code as in r06m): rocprofv3
# kernel statistics of the headline command with the pair kernels queued (no
# overlapping launches, so the plain average is the per-launch time) and of
# the LD-block command; bench lines C4 (default, CPU baseline), C4 20/5, LD
# blocks, C2, C5, rank 0's 1/8 and 1/4 shards
out=gpurun_out/r06r; mkdir -p $out; export TMPDIR=/tmp
WLD_PIPE_SERIALIZE=pair tools/gpu_step.sh 300 $out/prof_c4q.log rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c4q -o c4q -- python3 bench.py --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $out/prof_ldb.log rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_ldb -o ldb -- python3 bench.py --data ldblocks --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py || exit $?
tools/gpu_step.sh 200 $out/bench_c4_20_5.log python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $out/bench_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c2.log python bench.py --config c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 400 $out/bench_c5.log python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/shard8.log python bench.py --rehearse-dist --rehearse-shard 8 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/shard4.log python bench.py --rehearse-dist --rehearse-shard 4 --no-cpu-baseline || exit $?
echo done
