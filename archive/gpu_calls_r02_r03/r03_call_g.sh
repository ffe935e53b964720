#!/bin/bash
# round-3 GPU call G: the chunk scan fused into the screen's / candidate
# launch's last workgroup: the parity files, then the N>1 rehearsals and benches
out=gpurun_out/r03g; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 900 $out/tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_screen.py tests/test_gpu_refsums.py tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_dist.py -k "not full" || exit $?
tools/gpu_step.sh 200 $out/bench_c4_rehearse_s8.log python bench.py --rehearse-dist --rehearse-shard 8 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c4_rehearse_s4.log python bench.py --rehearse-dist --rehearse-shard 4 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c4.log python bench.py --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c4_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o s8 -- \
  python3 bench.py --rehearse-dist --rehearse-shard 8 --steps 100 --warmup 10 --no-cpu-baseline > $out/prof_s8.log 2>&1 || { echo "rocprof failed $?"; exit 1; }
echo done
