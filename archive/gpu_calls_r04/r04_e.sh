#!/bin/bash
# round-4 GPU call E: fp6 policy tests; A/B of the item kernels (C2, LD blocks)
# and of fp6 vs i8 on LD blocks; PMC passes and a kernel trace of the fp6
# screen at C4; bench lines
out=gpurun_out/r04e; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 900 $out/new_tests.txt python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_fp6.py tests/test_gpu_screen.py tests/test_gpu_refsums.py \
  tests/test_gpu_parity.py::test_progress_once_per_chunk_screened || exit $?
tools/gpu_step.sh 300 $out/ab_c2.txt python tools/ab_builds.py --config c2 --thr 0.0 --reps 20 --rounds 3 \
  item=weightedld_amd/libweightedld.so lds=build/exp/ldsitem/libweightedld.so nosel=build/exp/nosel/libweightedld.so || exit $?
WLD_AB_DATA=ldblocks tools/gpu_step.sh 400 $out/ab_ldb.txt python tools/ab_builds.py --config c4 --reps 10 --rounds 3 \
  fp6item=weightedld_amd/libweightedld.so@WLD_AB_OPTS=screen_fp6=2 i8item=weightedld_amd/libweightedld.so@WLD_AB_OPTS=screen_fp6=0 \
  fp6lds=build/exp/ldsitem/libweightedld.so@WLD_AB_OPTS=screen_fp6=2 nosel=build/exp/nosel/libweightedld.so@WLD_AB_OPTS=screen_fp6=0 || exit $?
tools/gpu_step.sh 300 $out/bench_c4.log python bench.py || exit $?
tools/gpu_step.sh 200 $out/bench_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c2.log python bench.py --config c2 --no-cpu-baseline || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c4 -o c4 -- \
  python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > $out/prof_c4.log 2>&1 || { echo "prof failed"; exit 1; }
bargs="--steps 5 --warmup 2 --settle-s 0 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $out/pmc_sq -o sq -- \
  python3 bench.py $bargs > $out/pmc_sq.log 2>&1 || { echo "pmc sq failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA \
  SQ_INSTS_LDS --output-format csv -d $out/pmc_lds -o lds -- python3 bench.py $bargs > $out/pmc_lds.log 2>&1 || { echo "pmc lds failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_fetch -o fetch -- \
  python3 bench.py $bargs > $out/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_write -o write -- \
  python3 bench.py $bargs > $out/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
echo done
