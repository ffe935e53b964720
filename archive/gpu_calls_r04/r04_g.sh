#!/bin/bash
# round-4 GPU call G: the whole -m gpu suite and smoke() on the tree with the
# item kernel's byte-convert operands; C2 and LD-block A/B against the
# per-element selects
out=gpurun_out/r04g; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 1000 $out/gpu_tests.txt python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests || exit $?
tools/gpu_step.sh 120 $out/smoke.txt python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
tools/gpu_step.sh 300 $out/ab_c2.txt python tools/ab_builds.py --config c2 --reps 30 --rounds 3 \
  cvt=weightedld_amd/libweightedld.so nocvt=build/exp/nocvt/libweightedld.so || exit $?
WLD_AB_DATA=ldblocks tools/gpu_step.sh 300 $out/ab_ldb.txt python tools/ab_builds.py --config c4 --reps 10 --rounds 3 \
  cvt=weightedld_amd/libweightedld.so nocvt=build/exp/nocvt/libweightedld.so || exit $?
tools/gpu_step.sh 200 $out/bench_c2_drain.log python bench.py --config c2 --no-cpu-baseline || exit $?
WLD_PIPE_DRAIN_ROWS=0 tools/gpu_step.sh 200 $out/bench_c2_nodrain.log python bench.py --config c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_ldb_drain.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
WLD_PIPE_DRAIN_ROWS=0 tools/gpu_step.sh 200 $out/bench_ldb_nodrain.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
echo done
