#!/bin/bash
# round-4 GPU call C: packed 16-row-block candidate items — targeted tests,
# A/B against the round-3 shape (whole tiles per workgroup, WLD_REF_ITEMS=0) at
# C2 and on LD blocks, PMC of both at C2, bench lines, kernel trace of C2
out=gpurun_out/r04c; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 900 $out/new_tests.txt python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py::test_cli_progress_bars tests/test_gpu_parity.py::test_progress_once_per_chunk_screened \
  tests/test_gpu_parity.py::test_progress_once_per_chunk_config2 tests/test_gpu_parity.py::test_contexts_on_one_stream \
  tests/test_gpu_refsums.py tests/test_gpu_screen.py || exit $?
grep -q " failed" $out/new_tests.txt && { echo "tests failed"; exit 1; }
tools/gpu_step.sh 300 $out/ab_c2.txt python tools/ab_builds.py --config c2 --thr 0.0 --reps 20 --rounds 3 \
  items=weightedld_amd/libweightedld.so r3=build/exp/r3items/libweightedld.so || exit $?
WLD_AB_DATA=ldblocks tools/gpu_step.sh 300 $out/ab_ldb.txt python tools/ab_builds.py --config c4 --reps 10 --rounds 3 \
  items=weightedld_amd/libweightedld.so r3=build/exp/r3items/libweightedld.so || exit $?
tools/gpu_step.sh 200 $out/bench_c2.log python bench.py --config c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_ldb.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
cd /tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $out/pmc_items -o items -- \
  python3 tools/ab_builds.py --child weightedld_amd/libweightedld.so --config c2 --thr 0.0 --reps 5 > $out/pmc_items.log 2>&1 || { echo "pmc items failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $out/pmc_r3 -o r3 -- \
  python3 tools/ab_builds.py --child build/exp/r3items/libweightedld.so --config c2 --thr 0.0 --reps 5 > $out/pmc_r3.log 2>&1 || { echo "pmc r3 failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c2 -o c2 -- \
  python3 bench.py --config c2 --steps 50 --warmup 5 --no-cpu-baseline > $out/prof_c2.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
