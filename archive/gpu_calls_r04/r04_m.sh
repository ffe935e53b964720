#!/bin/bash
# round-4 GPU call M: the chunk scan fused into full item runs, C2 bench
# lines with and without it (twice, interleaved)
out=gpurun_out/r04m; mkdir -p $out; export TMPDIR=/tmp
for r in a b; do
  tools/gpu_step.sh 200 $out/bench_c2_fused_$r.log python bench.py --config c2 --no-cpu-baseline || exit $?
  WLD_BENCH_OPTS="fused_scan=0" tools/gpu_step.sh 200 $out/bench_c2_sep_$r.log python bench.py --config c2 --no-cpu-baseline || exit $?
done
tools/gpu_step.sh 400 $out/ab_c4.txt python tools/ab_builds.py --config c4 --reps 20 --rounds 3 \
  base=weightedld_amd/libweightedld.so bmin=build/exp/bmin/libweightedld.so wg3=build/exp/wg3/libweightedld.so || exit $?
tools/gpu_step.sh 200 $out/ab_c4_rows.txt python tools/ab_builds.py --config 2000,4096,0.02 --reps 5 --rounds 1 \
  base=weightedld_amd/libweightedld.so bmin=build/exp/bmin/libweightedld.so || exit $?
echo done
