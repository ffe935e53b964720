#!/bin/bash
# round-4 GPU call P: where the fp6 screen's time goes at C4 (diagnostic
# builds, wrong results): 1 no epilogue, 2 also cache-resident copies,
# 3 also no MFMA
out=gpurun_out/r04p; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 400 $out/ab_c4.txt python tools/ab_builds.py --config c4 --reps 20 --rounds 3 \
  base=weightedld_amd/libweightedld.so d1=build/exp/f6diag1/libweightedld.so d2=build/exp/f6diag2/libweightedld.so \
  d3=build/exp/f6diag3/libweightedld.so || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $out/pmc_lds -o lds -- \
  python3 tools/ab_builds.py --child weightedld_amd/libweightedld.so --config c4 --reps 5 > $out/pmc_lds.log 2>&1 || { echo "pmc lds failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS \
  SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC --output-format csv -d $out/pmc_inst -o inst -- \
  python3 tools/ab_builds.py --child weightedld_amd/libweightedld.so --config c4 --reps 5 > $out/pmc_inst.log 2>&1 || { echo "pmc inst failed"; exit 1; }
echo done
