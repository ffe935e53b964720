#!/bin/bash
# round-3 GPU call H: fused scan without ticket traffic when no candidate;
# pipeline depth A/B on rank 0's 1/8 shard
out=gpurun_out/r03h; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 600 $out/tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_screen.py tests/test_gpu_refsums.py tests/test_gpu_dist.py -k "not full" || exit $?
for d in 2 3 4; do
tools/gpu_step.sh 200 $out/s8_d$d.log python bench.py --rehearse-dist --rehearse-shard 8 --pipe-depth $d --no-cpu-baseline || exit $?
done
tools/gpu_step.sh 200 $out/bench_c4.log python bench.py --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c4_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o s8 -- \
  python3 bench.py --rehearse-dist --rehearse-shard 8 --steps 100 --warmup 10 --no-cpu-baseline > $out/prof_s8.log 2>&1 || { echo "rocprof failed $?"; exit 1; }
echo done
