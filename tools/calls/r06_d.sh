#!/bin/bash
# round-6 GPU call D: m0-clobber A/B (fp6 C4, i8 LD blocks, 1/8 shard); the
# in-tree library's bench lines (C4 headline, LD blocks, the rehearsed 1/8
# shard twice) and the rocprofv3 kernel statistics of the headline command
out=gpurun_out/r06d; mkdir -p $out; export TMPDIR=/tmp
B="cur=weightedld_amd/libweightedld.so m0=build/exp/m0/libweightedld.so"
tools/gpu_step.sh 300 $out/ab_c4.log python tools/ab_builds.py --config c4 --reps 30 --rounds 3 $B || exit $?
WLD_AB_DATA=ldblocks tools/gpu_step.sh 300 $out/ab_ldb.log python tools/ab_builds.py --config c4 --reps 20 --rounds 3 $B || exit $?
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py || exit $?
tools/gpu_step.sh 300 $out/bench_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/shard8_a.log python bench.py --rehearse-dist --rehearse-shard 8 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/shard8_b.log python bench.py --rehearse-dist --rehearse-shard 8 --no-cpu-baseline || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_step.sh 300 $out/prof_c4.log rocprofv3 --kernel-trace --stats -d $out/prof_c4 -o c4 -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline || exit $?
echo done
