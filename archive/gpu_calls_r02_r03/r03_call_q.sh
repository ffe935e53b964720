#!/bin/bash
# round-3 GPU call Q: lib.rs-order screen policy test; N=1 loop with three
# contexts (overlapping screens) vs two queued with wld_run_after
out=gpurun_out/r03q; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 400 $out/tests.log python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_refsums.py -k "policy" || exit $?
for rep in 1 2; do
tools/gpu_step.sh 200 $out/c4_d3_0_r$rep.log python bench.py --no-cpu-baseline || exit $?
WLD_PIPE_SERIALIZE=pair tools/gpu_step.sh 200 $out/c4_d2_pair_r$rep.log python bench.py --pipe-depth 2 --no-cpu-baseline || exit $?
done
tools/gpu_step.sh 200 $out/ldb_d3_0.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
WLD_PIPE_SERIALIZE=pair tools/gpu_step.sh 200 $out/ldb_d2_pair.log python bench.py --data ldblocks --pipe-depth 2 --no-cpu-baseline || exit $?
echo done
