#!/bin/bash
# round-3 GPU call AJ: the candidate launch on a small grid where the one-plane
# screen's history over the same chunk range says its list will be empty
# (MfmaLaunch::cand_grid): the new history test first, then the GPU suite,
# then bench A/B against HEAD's library (in-tree .so swapped): C4 N=1 and the
# rehearsed 1/8 shard (the per-rank work at N=8)
out=gpurun_out/r03aj; mkdir -p $out; export TMPDIR=/tmp
cp build/exp/grid/libweightedld.so weightedld_amd/libweightedld.so
tools/gpu_step.sh 300 $out/test_history.txt python -u -m pytest tests/test_gpu_refsums.py -m gpu -x -q -rf --timeout 200 --timeout-method thread -k empty_candidate || exit $?
grep -q " passed" $out/test_history.txt && ! grep -q " failed" $out/test_history.txt || { echo "history test not green"; exit 1; }
tools/gpu_step.sh 900 $out/gpu_tests.txt python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread || exit $?
for r in 1 2; do
  for b in head grid; do
    cp build/exp/$b/libweightedld.so weightedld_amd/libweightedld.so
    tools/gpu_step.sh 200 $out/bench_${b}_$r.log python bench.py --no-cpu-baseline || exit $?
    tools/gpu_step.sh 200 $out/shard8_${b}_$r.log python bench.py --no-cpu-baseline --rehearse-dist --rehearse-shard 8 --steps 400 --warmup 40 || exit $?
  done
done
cp build/exp/grid/libweightedld.so weightedld_amd/libweightedld.so
echo done
