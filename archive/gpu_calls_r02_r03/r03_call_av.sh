#!/bin/bash
# round-3 GPU call AV: the final tree (XCD super-block size chosen from the L2
# footprint) — the -m gpu suite, smoke(), the default bench (CPU baseline and
# oracle row check), 20/5, LD blocks, C5, C2, the rehearsed 1/8 shard, and
# rocprofv3 kernel stats of the default bench
out=gpurun_out/r03av; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 900 $out/gpu_tests.txt python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread || exit $?
tools/gpu_step.sh 200 $out/smoke.txt python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py || exit $?
tools/gpu_step.sh 200 $out/bench_c4_20_5.log python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $out/bench_c5.log python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c2.log python bench.py --config c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/shard8.log python bench.py --no-cpu-baseline --rehearse-dist --rehearse-shard 8 --steps 400 --warmup 40 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o c4 -- \
  python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > $out/prof_c4.log 2>&1 || { echo "rocprof failed $?"; exit 1; }
echo done
