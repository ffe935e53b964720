#!/bin/bash
# round-4 GPU call X: PMC passes on the final fp6 screen at C4 (vector issue
# vs matrix pipe), each pass its own run
out=gpurun_out/r04x; mkdir -p $out; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
  SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d $out/pmc_issue -o issue -- \
  python3 tools/ab_builds.py --child weightedld_amd/libweightedld.so --config c4 --reps 5 > $out/pmc_issue.log 2>&1 || { echo "pmc issue failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU \
  --output-format csv -d $out/pmc_coexec -o coexec -- \
  python3 tools/ab_builds.py --child weightedld_amd/libweightedld.so --config c4 --reps 5 > $out/pmc_coexec.log 2>&1 || { echo "pmc coexec failed"; exit 0; }
echo done
