#!/bin/bash
# round-4 GPU call T (tree at the end of the round): the whole -m gpu suite,
# smoke(), the headline bench line, its rocprofv3 kernel summary, and the LD
# block and C2 lines
out=gpurun_out/r04t; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 700 $out/gpu_tests.txt python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests || exit $?
tools/gpu_step.sh 120 $out/smoke.txt python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
tools/gpu_step.sh 200 $out/bench_c4.log python bench.py || exit $?
tools/gpu_step.sh 200 $out/prof_c4.log rocprofv3 --kernel-trace --stats -d $out/prof_c4 -o c4 -- python3 bench.py --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
tools/gpu_step.sh 150 $out/bench_c2.log python bench.py --config c2 --no-cpu-baseline || exit $?
echo done
