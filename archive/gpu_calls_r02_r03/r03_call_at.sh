#!/bin/bash
# round-3 GPU call AT: the tree with 16x16 XCD super-blocks — the -m gpu suite,
# smoke(), the default bench (CPU baseline, oracle row check), 20/5, LD blocks,
# C5, the rehearsed 1/8 shard, rocprofv3 kernel stats, and the FETCH_SIZE /
# WRITE_SIZE passes of the C4 screen (profiles/traffic.json)
out=gpurun_out/r03at; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 900 $out/gpu_tests.txt python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread || exit $?
tools/gpu_step.sh 200 $out/smoke.txt python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py || exit $?
tools/gpu_step.sh 200 $out/bench_c4_20_5.log python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $out/bench_c5.log python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/shard8.log python bench.py --no-cpu-baseline --rehearse-dist --rehearse-shard 8 --steps 400 --warmup 40 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o c4 -- \
  python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > $out/prof_c4.log 2>&1 || { echo "rocprof failed $?"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $out/pmc/fetch -o fetch -- \
  python3 bench.py --no-pipeline --steps 10 --warmup 2 --no-cpu-baseline > $out/pmc_fetch.log 2>&1 || { echo "pmc fetch failed $?"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $out/pmc/write -o write -- \
  python3 bench.py --no-pipeline --steps 10 --warmup 2 --no-cpu-baseline > $out/pmc_write.log 2>&1 || { echo "pmc write failed $?"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $out/pmc/l2 -o l2 -- \
  python3 bench.py --no-pipeline --steps 10 --warmup 2 --no-cpu-baseline > $out/pmc_l2.log 2>&1 || { echo "pmc l2 failed $?"; exit 1; }
echo done
