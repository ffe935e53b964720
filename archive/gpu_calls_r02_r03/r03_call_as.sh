#!/bin/bash
# round-3 GPU call AS: XCD super-block size kS of the screen's launch order,
# full bench lines interleaved (8 shipped; 12, 16, 24 as -DWLD_XCD_SB builds),
# three passes, and rank 0's 1/8 shard for 8 vs 16
out=gpurun_out/r03as; mkdir -p $out; export TMPDIR=/tmp
cp weightedld_amd/libweightedld.so /tmp/lib_main.so
use() { if [ $1 = main ]; then cp /tmp/lib_main.so weightedld_amd/libweightedld.so; else cp build/exp/$1/libweightedld.so weightedld_amd/libweightedld.so; fi; }
for pass in 1 2 3; do for v in main sb12 sb16 sb24; do
use $v
tools/gpu_step.sh 200 $out/p${pass}_c4_$v.log python bench.py --no-cpu-baseline || { cp /tmp/lib_main.so weightedld_amd/libweightedld.so; exit 1; }
done; done
for pass in 1 2; do for v in main sb16; do
use $v
tools/gpu_step.sh 200 $out/p${pass}_shard8_$v.log python bench.py --no-cpu-baseline --rehearse-dist --rehearse-shard 8 --steps 400 --warmup 40 || { cp /tmp/lib_main.so weightedld_amd/libweightedld.so; exit 1; }
done; done
cp /tmp/lib_main.so weightedld_amd/libweightedld.so
echo done
