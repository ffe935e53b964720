#!/bin/bash
# round-5 GPU call I: PMC passes (issue / waits+LDS) on the tile-pair fp6
# screen (fp4 B) and the round-4 kernel at C4, each pass its own run
out=gpurun_out/r05i; mkdir -p $out; export TMPDIR=/tmp
for b in old pairs; do
  lib=build/exp/$b/libweightedld.so; [ $b = pairs ] && lib=weightedld_amd/libweightedld.so
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
    SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d $out/${b}_issue -o issue -- \
    python3 tools/ab_builds.py --child $lib --config c4 --reps 5 > $out/${b}_issue.log 2>&1 || { echo "pmc issue $b failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS \
    --output-format csv -d $out/${b}_wait -o wait -- \
    python3 tools/ab_builds.py --child $lib --config c4 --reps 5 > $out/${b}_wait.log 2>&1 || { echo "pmc wait $b failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC \
    SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS --output-format csv -d $out/${b}_misc -o misc -- \
    python3 tools/ab_builds.py --child $lib --config c4 --reps 5 > $out/${b}_misc.log 2>&1 || { echo "pmc misc $b failed"; exit 0; }
done
for b in old pairs; do echo "== $b"; python3 tools/pmc_kernels.py $(find $out/${b}_* -name "*counter_collection.csv") --match fp6; done > $out/summary.txt
cat $out/summary.txt
echo done
