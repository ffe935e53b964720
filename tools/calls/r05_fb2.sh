#!/bin/bash
# round-5 final call B (wide-wave screen tree): bench lines (headline with the CPU baseline, the
# driver's 20/5, LD blocks, C2, C5, rehearsed 1/8 and 1/4 shards, 2 ranks),
# rocprofv3 kernel statistics of the headline command, PMC traffic passes,
# first-pass timings
out=gpurun_out/r05_final2; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py || exit $?
tools/gpu_step.sh 120 $out/bench_c4_20_5.log python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c2.log python bench.py --config c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c5.log python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_shard8.log python bench.py --rehearse-dist --rehearse-shard 8 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_shard4.log python bench.py --rehearse-dist --rehearse-shard 4 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_gpus2.log python bench.py --gpus 2 --collectives gloo --check-steps 2 --no-cpu-baseline || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c4 -o c4 -- \
  python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > $out/prof_c4.log 2>&1 || { echo "prof failed"; exit 1; }
bargs="--steps 5 --warmup 2 --settle-s 0 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_fetch -o fetch -- \
  python3 bench.py $bargs > $out/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_write -o write -- \
  python3 bench.py $bargs > $out/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_l2 -o l2 -- \
  python3 bench.py $bargs > $out/pmc_l2.log 2>&1 || { echo "pmc l2 failed"; exit 1; }
tools/gpu_step.sh 200 $out/first_rand.log python3 tools/first_pass.py random 0.05 || exit $?
tools/gpu_step.sh 200 $out/first_ldb.log python3 tools/first_pass.py ldblocks 0.05 || exit $?
echo done
