#!/bin/bash
# round-3 GPU call E: N>1 rehearsals (whole C4 and rank 0's 1/8 shard through
# an RCCL group of one) and their kernel traces
out=gpurun_out/r03e; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 200 $out/bench_c4_rehearse.log python bench.py --rehearse-dist --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c4_rehearse_s8.log python bench.py --rehearse-dist --rehearse-shard 8 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c4_rehearse_s4.log python bench.py --rehearse-dist --rehearse-shard 4 --no-cpu-baseline || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o s8 -- \
  python3 bench.py --rehearse-dist --rehearse-shard 8 --steps 100 --warmup 10 --no-cpu-baseline > $out/prof_s8.log 2>&1 || { echo "rocprof failed $?"; exit 1; }
echo done
