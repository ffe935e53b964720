#!/bin/bash
# Round-end check of the committed tree: the -m gpu suite, smoke(), the N>1
# step path rehearsed through an RCCL group of one (C4, C2), and the C4 line
# at thr 0.01 (the screen's two-plane tier).  -> gpurun_out/TAG/
out=gpurun_out/${1:-r02f}; mkdir -p $out
export TMPDIR=/tmp
tools/gpu_step.sh 700 $out/gpu_tests.txt python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread || exit $?
tools/gpu_step.sh 120 $out/smoke.txt python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
tools/gpu_step.sh 200 $out/bench_c4_rehearse.log python bench.py --rehearse-dist --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c2_rehearse.log python bench.py --rehearse-dist --config c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c4_thr001.log python bench.py --thr 0.01 --steps 50 --warmup 5 --no-cpu-baseline || exit $?
echo done
