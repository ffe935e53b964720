#!/bin/bash
# round-4 GPU call U (tree at the end of the round, after removing the A/B
# switches and the unused one-slot kernel variant, and with the CPU baseline
# at N=1 only): the whole -m gpu suite, smoke(), the headline bench line and
# its rocprofv3 summary, the LD-block and C2 lines, the rehearsed 1/8 shard
out=gpurun_out/r04u; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 600 $out/gpu_tests.txt python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests || exit $?
tools/gpu_step.sh 120 $out/smoke.txt python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
tools/gpu_step.sh 150 $out/bench_c4.log python bench.py || exit $?
tools/gpu_step.sh 150 $out/prof_c4.log rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c4 -o c4 -- python3 bench.py --no-cpu-baseline || exit $?
tools/gpu_step.sh 120 $out/bench_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
tools/gpu_step.sh 100 $out/bench_c2.log python bench.py --config c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 120 $out/bench_shard8.log python bench.py --rehearse-dist --rehearse-shard 8 --no-cpu-baseline || exit $?
echo done
