#!/bin/bash
# round-6 GPU call M (re-entry after the container was re-created): the
# B-rolled screens' tree — the whole GPU suite and smoke, then the headline
# bench, LD blocks, C2, the 1/8 shard and the rocprofv3 kernel statistics
out=gpurun_out/r06m; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 1000 $out/tests.log python3 -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests -m gpu || exit $?
tools/gpu_step.sh 120 $out/smoke.txt python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py || exit $?
tools/gpu_step.sh 300 $out/bench_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c2.log python bench.py --config c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/shard8.log python bench.py --rehearse-dist --rehearse-shard 8 --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $out/prof_c4.log rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c4 -o c4 -- python3 bench.py --no-cpu-baseline || exit $?
echo done
