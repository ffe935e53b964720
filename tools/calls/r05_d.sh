#!/bin/bash
# round-5 GPU call D: PMC passes (issue / waits+LDS) on the three fp6 screens
# at C4 (one-at-a-time harness), each pass its own run
out=gpurun_out/r05d; mkdir -p $out; export TMPDIR=/tmp
for b in old alds areg; do
  lib=build/exp/$b/libweightedld.so; [ $b = areg ] && lib=weightedld_amd/libweightedld.so
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
    SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d $out/${b}_issue -o issue -- \
    python3 tools/ab_builds.py --child $lib --config c4 --reps 5 > $out/${b}_issue.log 2>&1 || { echo "pmc issue $b failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS \
    --output-format csv -d $out/${b}_wait -o wait -- \
    python3 tools/ab_builds.py --child $lib --config c4 --reps 5 > $out/${b}_wait.log 2>&1 || { echo "pmc wait $b failed"; exit 1; }
done
for b in old alds areg; do echo "== $b"; python3 tools/pmc_kernels.py $(find $out/${b}_issue $out/${b}_wait -name "*counter_collection.csv") --match fp6; done > $out/summary.txt
cat $out/summary.txt
echo done
