#!/bin/bash
# round-6 GPU call AK (final product tree: LDS-staged candidate items and B rows, the
# batched gather): the whole GPU suite and smoke; the driver's bench command
# and the default one; LD blocks, C2, C5, rank 0's 1/8 shard; the headline
# command under rocprofv3 with the passes queued
out=gpurun_out/r06ak; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 1000 $out/tests.log python3 -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests -m gpu || exit $?
tools/gpu_step.sh 120 $out/smoke.txt python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py || exit $?
tools/gpu_step.sh 200 $out/bench_c4_20_5.log python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $out/bench_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c2.log python bench.py --config c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 400 $out/bench_c5.log python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/shard8.log python bench.py --rehearse-dist --rehearse-shard 8 --no-cpu-baseline || exit $?
WLD_PIPE_SERIALIZE=pair tools/gpu_step.sh 300 $out/prof_c4q.log rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c4q -o c4q -- python3 bench.py --no-cpu-baseline || exit $?
echo done
