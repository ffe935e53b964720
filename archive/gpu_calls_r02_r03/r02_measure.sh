#!/bin/bash
# One GPU call for the round-2 measurements of the committed tree:
# GPU tests, bench lines (C4 pipelined + not, C2, C5, unweighted, wide weights,
# f32 fallback) and the rocprofv3 kernel trace/stats of the non-pipelined C4 bench.
#   tools/calls/r02_measure.sh TAG   -> gpurun_out/TAG/...
out=gpurun_out/${1:-r02m}
mkdir -p $out
export TMPDIR=/tmp
tools/gpu_step.sh 600 $out/gpu_tests.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread || exit $?
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py || exit $?
tools/gpu_step.sh 200 $out/bench_c4_nopipe.log python bench.py --no-pipeline --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c2.log python bench.py --config c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c4_unweighted.log python bench.py --unweighted --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c4_wide.log python bench.py --wide-weights --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c4_valu.log python bench.py --kernel valu --steps 5 --warmup 1 --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $out/bench_c5.log python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c4_rehearse.log python bench.py --rehearse-dist --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c4_rehearse_s8.log python bench.py --rehearse-dist --rehearse-shard 8 --no-cpu-baseline || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o c4_nopipe -- \
  python3 bench.py --no-pipeline --steps 50 --warmup 5 --no-cpu-baseline > $out/prof.log 2>&1 || { echo "rocprof failed $?"; exit 1; }
echo done
