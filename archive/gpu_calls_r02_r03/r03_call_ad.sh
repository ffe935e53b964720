#!/bin/bash
# round-3 GPU call AD: BASELINE config 5 (the north star's 8-GPU config) per
# rank: rank 0's 1/8 shard through the N>1 step path, and the whole C5 step
out=gpurun_out/r03ad; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 400 $out/c5_rehearse_s8.log python bench.py --config c5 --rehearse-dist --rehearse-shard 8 --steps 50 --warmup 5 --no-cpu-baseline || exit $?
tools/gpu_step.sh 400 $out/c5_rehearse.log python bench.py --config c5 --rehearse-dist --steps 20 --warmup 3 --no-cpu-baseline || exit $?
echo done
