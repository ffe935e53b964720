#!/bin/bash
# round-5 GPU call AJ: the tile-pair fp6 screen reading B's minor-bit planes from
# LDS (made once by frag6_kernel) instead of masking per wave: A/B at C4 and C5,
# its vector-instruction count (PMC), and the fp6 / screen suites on it
out=gpurun_out/r05aj; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 500 $out/ab_c4.log python3 tools/ab_builds.py --config c4 --reps 10 --rounds 3 \
  base=weightedld_amd/libweightedld.so bmin=build/exp/bmin/libweightedld.so || exit 1
tools/gpu_step.sh 400 $out/ab_c5.log python3 tools/ab_builds.py --config c5 --reps 4 --rounds 2 \
  base=weightedld_amd/libweightedld.so bmin=build/exp/bmin/libweightedld.so || exit 1
for b in base bmin; do
  lib=weightedld_amd/libweightedld.so; [ $b = bmin ] && lib=build/exp/bmin/libweightedld.so
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d $out/pmc_$b -o pmc -- python3 tools/ab_builds.py --child $lib --config c4 --reps 5 > $out/pmc_$b.log 2>&1 || { echo "pmc $b failed"; exit 1; }
done
for b in base bmin; do echo "== $b"; python3 tools/pmc_kernels.py $(find $out/pmc_$b -name "*counter_collection.csv") --match fp6; done > $out/pmc_summary.txt
tools/gpu_step.sh 600 $out/tests_bmin.log env WLD_LIB_PATH=build/exp/bmin/libweightedld.so python3 -u -m pytest -x -q \
  --timeout 300 --timeout-method thread tests/test_gpu_fp6.py tests/test_gpu_screen.py -k "not full_size" || exit 1
echo done
