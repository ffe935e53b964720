#!/bin/bash
# round-6 GPU call X: full runs (C2) on the LDS-staged item path (no A share,
# five workgroups per CU) against the A-share path at six: A/B at C2
out=gpurun_out/r06x; mkdir -p $out; export TMPDIR=/tmp
B="base=weightedld_amd/libweightedld.so fs5=build/exp/fs5/libweightedld.so"
tools/gpu_step.sh 300 $out/ab_c2.log python tools/ab_builds.py --config c2 --reps 40 --rounds 5 $B || exit $?
WLD_LIB_PATH=build/exp/fs5/libweightedld.so tools/gpu_step.sh 200 $out/bench_c2_fs5.log python bench.py --config c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c2_base.log python bench.py --config c2 --no-cpu-baseline || exit $?
echo done
