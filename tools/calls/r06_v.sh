#!/bin/bash
# round-6 GPU call V: LDS-staged candidate items (five workgroups per CU) as
# the default — the whole GPU suite and smoke, then LD blocks (twice), C4,
# and the LD-block command's rocprofv3 statistics with whole passes queued
out=gpurun_out/r06v; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 1000 $out/tests.log python3 -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests -m gpu || exit $?
tools/gpu_step.sh 120 $out/smoke.txt python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
tools/gpu_step.sh 300 $out/bench_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $out/bench_ldb_b.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py --no-cpu-baseline || exit $?
WLD_PIPE_SERIALIZE=1 tools/gpu_step.sh 300 $out/prof_ldb.log rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_ldb -o ldb -- python3 bench.py --data ldblocks --no-cpu-baseline || exit $?
echo done
