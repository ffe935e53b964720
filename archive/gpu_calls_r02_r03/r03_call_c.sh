#!/bin/bash
# round-3 GPU call C: bench lines (default 200/20, the driver's 20/5, LD blocks in
# both summation modes) and a rocprofv3 kernel trace of the 20/5 command
out=gpurun_out/${1:-r03c}; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py || exit $?
tools/gpu_step.sh 200 $out/bench_c4_20_5.log python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $out/bench_c4_ldblocks.log python bench.py --data ldblocks || exit $?
tools/gpu_step.sh 200 $out/bench_c4_ldblocks_exact.log python bench.py --data ldblocks --exact-sums --no-cpu-baseline || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o c4_20_5 -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/prof_20_5.log 2>&1 || { echo "rocprof failed $?"; exit 1; }
tools/gpu_step.sh 400 $out/pk_hazard.txt python -u tools/probes/pk_hazard.py --reps 1 || exit $?
tools/gpu_step.sh 300 $out/pk_hazard_small.txt python -u tools/probes/pk_hazard.py --small || exit $?
echo done
