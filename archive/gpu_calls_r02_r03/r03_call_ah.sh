#!/bin/bash
# round-3 GPU call AH: chunk scan with the totals loaded all at once and kept in
# registers, candidate launches' idle workgroups skipping cand_prefix: the GPU
# suite on that build, then bench A/B (in-tree .so swapped) against HEAD's
# library, two contexts with wld_run_after (default) and both on one stream
out=gpurun_out/r03ah; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 900 $out/gpu_tests.txt python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread || exit $?
grep -q " passed" $out/gpu_tests.txt && ! grep -q " failed" $out/gpu_tests.txt || { echo "tests not green"; exit 1; }
for r in 1 2; do
  for b in head scan; do
    cp build/exp/$b/libweightedld.so weightedld_amd/libweightedld.so
    tools/gpu_step.sh 200 $out/bench_${b}_pair_$r.log python bench.py --no-cpu-baseline || exit $?
    WLD_PIPE_SERIALIZE=stream tools/gpu_step.sh 200 $out/bench_${b}_stream_$r.log python bench.py --no-cpu-baseline || exit $?
  done
done
cp build/exp/scan/libweightedld.so weightedld_amd/libweightedld.so
echo done
