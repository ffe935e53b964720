#!/bin/bash
# (experiment: the split was measured slower and reverted)
# round-3 GPU call AX: heavy candidate tiles split into two work items (a rows
# 0-31 / 32-63): the screen, ref-sums and parity GPU tests, then the LD-block
# line against build/exp/nosplit (-DWLD_CAND_SPLIT=0), interleaved, 3 passes
out=gpurun_out/r03ax; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 600 $out/gpu_tests.txt python -u -m pytest tests/test_gpu_refsums.py tests/test_gpu_screen.py tests/test_gpu_parity.py -m gpu -q -rf --timeout 300 --timeout-method thread || exit $?
grep -q " passed" $out/gpu_tests.txt && ! grep -q " failed" $out/gpu_tests.txt || { echo "tests failed"; exit 1; }
cp weightedld_amd/libweightedld.so /tmp/lib_main.so
use() { if [ $1 = main ]; then cp /tmp/lib_main.so weightedld_amd/libweightedld.so; else cp build/exp/$1/libweightedld.so weightedld_amd/libweightedld.so; fi; }
for pass in 1 2 3; do for v in main nosplit; do
use $v
tools/gpu_step.sh 200 $out/p${pass}_ldb_$v.log python bench.py --data ldblocks --no-cpu-baseline || { cp /tmp/lib_main.so weightedld_amd/libweightedld.so; exit 1; }
done; done
cp /tmp/lib_main.so weightedld_amd/libweightedld.so
tools/gpu_step.sh 300 $out/ldb_rows.log python bench.py --data ldblocks || exit $?
echo done
