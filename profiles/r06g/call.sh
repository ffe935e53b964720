#!/bin/bash
# round-6 GPU call G: the candidate launch sized from the last pass (A/B
# against the fixed grid) at C4 and on LD blocks; then the whole GPU suite on
# the in-tree library, smoke, and the headline bench line
out=gpurun_out/r06g; mkdir -p $out; export TMPDIR=/tmp
B="hint=weightedld_amd/libweightedld.so nohint=build/exp/nohint/libweightedld.so"
tools/gpu_step.sh 300 $out/ab_c4.log python tools/ab_builds.py --config c4 --reps 30 --rounds 3 $B || exit $?
WLD_AB_DATA=ldblocks tools/gpu_step.sh 300 $out/ab_ldb.log python tools/ab_builds.py --config c4 --reps 20 --rounds 3 $B || exit $?
tools/gpu_step.sh 1000 $out/tests.log python3 -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests -m gpu || exit $?
tools/gpu_step.sh 120 $out/smoke.txt python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py || exit $?
echo done
