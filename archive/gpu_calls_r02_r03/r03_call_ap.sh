#!/bin/bash
# (the "screen" mode and wld_set_screen_stream were reverted after this call; the tree it ran is described in DESIGN.md §6, "Between screens")
# round-3 GPU call AP: screens of the N=1 pipelined loop on one stream
# (wld_set_screen_stream, WLD_PIPE_SERIALIZE=screen) against the default
# (wld_run_after, "pair"): the stream tests, then C4 and LD blocks A/B
# interleaved, three passes, and a kernel trace of the new mode
out=gpurun_out/r03ap; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 300 $out/gpu_tests.txt python -u -m pytest tests/test_gpu_parity.py -m gpu -v -rf --timeout 120 --timeout-method thread -k "stream or async or run_after or pipelined" || exit $?
grep -q " passed" $out/gpu_tests.txt && ! grep -q " failed" $out/gpu_tests.txt || { echo "tests failed"; exit 1; }
for pass in 1 2 3; do for m in pair screen; do
WLD_PIPE_SERIALIZE=$m tools/gpu_step.sh 200 $out/p${pass}_c4_$m.log python bench.py --no-cpu-baseline || exit $?
done; done
for m in pair screen; do
WLD_PIPE_SERIALIZE=$m tools/gpu_step.sh 200 $out/ldb_$m.log python bench.py --no-cpu-baseline --data ldblocks || exit $?
done
export WLD_PIPE_SERIALIZE=screen
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o c4_screen -- \
  python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > $out/prof_c4.log 2>&1 || { echo "rocprof failed $?"; exit 1; }
echo done
