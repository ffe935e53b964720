#!/bin/bash
# round-3 GPU call T: contexts on one stream (wld_set_stream): test, then the
# N=1 loop A/B (one stream vs wld_run_after events), C4 default
out=${OUT:-gpurun_out/r03t}; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 900 $out/tests.log python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_dist.py || exit $?
for rep in 1 2 3; do
WLD_PIPE_SERIALIZE=stream tools/gpu_step.sh 200 $out/c4_stream_r$rep.log python bench.py --no-cpu-baseline || exit $?
WLD_PIPE_SERIALIZE=pair tools/gpu_step.sh 200 $out/c4_pair_r$rep.log python bench.py --no-cpu-baseline || exit $?
done
echo done
