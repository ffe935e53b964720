#!/bin/bash
# round-3 GPU call AU: C5 and C2 with 16x16 XCD super-blocks (shipped) vs 8x8
# (build/exp/sb8), interleaved, two passes
out=gpurun_out/r03au; mkdir -p $out; export TMPDIR=/tmp
cp weightedld_amd/libweightedld.so /tmp/lib_main.so
use() { if [ $1 = main ]; then cp /tmp/lib_main.so weightedld_amd/libweightedld.so; else cp build/exp/$1/libweightedld.so weightedld_amd/libweightedld.so; fi; }
for pass in 1 2; do for v in main sb8; do
use $v
tools/gpu_step.sh 300 $out/p${pass}_c5_$v.log python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline || { cp /tmp/lib_main.so weightedld_amd/libweightedld.so; exit 1; }
tools/gpu_step.sh 300 $out/p${pass}_c4_$v.log python bench.py --no-cpu-baseline || { cp /tmp/lib_main.so weightedld_amd/libweightedld.so; exit 1; }
done; done
cp /tmp/lib_main.so weightedld_amd/libweightedld.so
echo done
