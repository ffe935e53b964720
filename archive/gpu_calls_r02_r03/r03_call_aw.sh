#!/bin/bash
# round-3 GPU call AW: C5's XCD super-block size (8 shipped; 4, 6, 11 as
# builds of the same rule with another large-NP size), interleaved, two passes
out=gpurun_out/r03aw; mkdir -p $out; export TMPDIR=/tmp
cp weightedld_amd/libweightedld.so /tmp/lib_main.so
use() { if [ $1 = main ]; then cp /tmp/lib_main.so weightedld_amd/libweightedld.so; else cp build/exp/$1/libweightedld.so weightedld_amd/libweightedld.so; fi; }
for pass in 1 2; do for v in main c5sb4 c5sb6 c5sb11; do
use $v
tools/gpu_step.sh 300 $out/p${pass}_c5_$v.log python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline || { cp /tmp/lib_main.so weightedld_amd/libweightedld.so; exit 1; }
done; done
cp /tmp/lib_main.so weightedld_amd/libweightedld.so
echo done
