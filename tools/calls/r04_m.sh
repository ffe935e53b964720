#!/bin/bash
# round-4 GPU call M: the chunk scan fused into full item runs, C2 bench
# lines with and without it (twice, interleaved)
out=gpurun_out/r04m; mkdir -p $out; export TMPDIR=/tmp
for r in a b; do
  tools/gpu_step.sh 200 $out/bench_c2_fused_$r.log python bench.py --config c2 --no-cpu-baseline || exit $?
  WLD_BENCH_OPTS="fused_scan=0" tools/gpu_step.sh 200 $out/bench_c2_sep_$r.log python bench.py --config c2 --no-cpu-baseline || exit $?
done
echo done
