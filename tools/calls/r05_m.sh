#!/bin/bash
# round-5 GPU call M: is the fp6 screen held by the clock (power)? The same
# C4 screen on Henikoff vs unit weights (same instruction stream, less operand
# toggling): kernel time and GRBM_GUI_ACTIVE (clock) per launch
out=gpurun_out/r05m; mkdir -p $out; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --output-format csv \
  -d $out/henikoff -o pmc -- python3 tools/ab_builds.py --child weightedld_amd/libweightedld.so --config c4 --reps 10 \
  > $out/henikoff.log 2>&1 || { echo "pmc henikoff failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --output-format csv \
  -d $out/unit -o pmc -- python3 tools/ab_builds.py --child weightedld_amd/libweightedld.so --config c4 --reps 10 --unweighted \
  > $out/unit.log 2>&1 || { echo "pmc unit failed"; exit 1; }
for b in henikoff unit; do echo "== $b"; tail -1 $out/$b.log; python3 tools/pmc_kernels.py $(find $out/$b -name "*counter_collection.csv") --match fp6; done > $out/summary.txt
cat $out/summary.txt
