#!/bin/bash
# round-5 GPU call F: where the fp6 screen's loop time goes (diagnostic builds,
# timing only, rows wrong): no epilogue; + cache-resident operand images;
# no MFMA (operands still read from LDS); both
out=gpurun_out/r05f; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 500 $out/ab_c4.log python3 tools/ab_builds.py --config c4 --reps 10 --rounds 3 \
  alds_top=build/exp/alds_top/libweightedld.so noepi=build/exp/d_noepi_alds/libweightedld.so \
  noepi_res=build/exp/d_noepi_res_alds/libweightedld.so nomfma=build/exp/d_nomfma_alds/libweightedld.so \
  nomfma_res=build/exp/d_nomfma_res_alds/libweightedld.so || exit 1
echo done
