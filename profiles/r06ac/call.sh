#!/bin/bash
# round-6 GPU call AC: the row gather visiting only the (chunk, slice) items
# of chunks with rows, their emptiness read 256 at a time (in-tree build),
# against HEAD's one round trip per item: parity/refsums tests on it, then
# bench.py on LD blocks (order phase and step) and C2, alternating builds
out=gpurun_out/r06ac; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 900 $out/tests.log python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_refsums.py -m gpu || exit $?
for i in 1 2; do
  WLD_LIB_PATH=build/exp/head/libweightedld.so tools/gpu_step.sh 300 $out/ldb_head_$i.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
  tools/gpu_step.sh 300 $out/ldb_new_$i.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
done
WLD_LIB_PATH=build/exp/head/libweightedld.so tools/gpu_step.sh 200 $out/c2_head.log python bench.py --config c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/c2_new.log python bench.py --config c2 --no-cpu-baseline || exit $?
echo done
