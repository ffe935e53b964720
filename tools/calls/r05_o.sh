#!/bin/bash
# round-5 GPU call O (mid-round tree): bench lines (headline with the CPU
# baseline, the driver's 20/5, LD blocks, C2, C5, rehearsed 1/8 shard),
# rocprofv3 kernel statistics of the headline command, PMC passes over the
# tile-pair fp6 screen (FETCH_SIZE, WRITE_SIZE, TCC hit/miss, SQ)
out=gpurun_out/r05o; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py || exit $?
tools/gpu_step.sh 120 $out/bench_c4_20_5.log python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c2.log python bench.py --config c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c5.log python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_shard8.log python bench.py --rehearse-dist --rehearse-shard 8 --no-cpu-baseline || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c4 -o c4 -- \
  python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > $out/prof_c4.log 2>&1 || { echo "prof failed"; exit 1; }
bargs="--steps 5 --warmup 2 --settle-s 0 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $out/pmc_sq -o sq -- \
  python3 bench.py $bargs > $out/pmc_sq.log 2>&1 || { echo "pmc sq failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_fetch -o fetch -- \
  python3 bench.py $bargs > $out/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_write -o write -- \
  python3 bench.py $bargs > $out/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_l2 -o l2 -- \
  python3 bench.py $bargs > $out/pmc_l2.log 2>&1 || { echo "pmc l2 failed"; exit 1; }

# the C2 item kernel's SIMD time
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d $out/pmc_c2 -o c2 -- \
  python3 bench.py --config c2 $bargs > $out/pmc_c2.log 2>&1 || { echo "pmc c2 failed"; exit 1; }
# where a fresh context's first pass spends its time (HIP API + kernel trace)
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $out/trace_first -o first -- \
  python3 tools/first_pass.py random 0.05 > $out/trace_first.log 2>&1 || { echo "trace failed"; exit 1; }
echo done
