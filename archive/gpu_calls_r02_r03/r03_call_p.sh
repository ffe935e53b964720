#!/bin/bash
# round-3 GPU call P: N=1 loop, three contexts with overlapping screens vs two
# queued with wld_run_after (C4 default and LD-block data)
out=gpurun_out/r03p; mkdir -p $out; export TMPDIR=/tmp
for rep in 1 2; do
tools/gpu_step.sh 200 $out/c4_d3_0_r$rep.log python bench.py --no-cpu-baseline || exit $?
WLD_PIPE_SERIALIZE=pair tools/gpu_step.sh 200 $out/c4_d2_pair_r$rep.log python bench.py --pipe-depth 2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/ldb_d3_0_r$rep.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
WLD_PIPE_SERIALIZE=pair tools/gpu_step.sh 200 $out/ldb_d2_pair_r$rep.log python bench.py --data ldblocks --pipe-depth 2 --no-cpu-baseline || exit $?
done
echo done
