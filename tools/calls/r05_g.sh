#!/bin/bash
# round-5 GPU call G: the fp6 screen's data skeleton (no MFMA, no epilogue,
# cache-resident images; timing only): all 18 LDS-DMA pieces per stage vs one
# per wave, with and without the per-stage barrier; and the MFMA loop with one
# piece per wave
out=gpurun_out/r05g; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 500 $out/ab_c4.log python3 tools/ab_builds.py --config c4 --reps 10 --rounds 3 \
  nm_res=build/exp/d_nomfma_res_alds/libweightedld.so nm_res_1dma=build/exp/d_nm_res_1dma/libweightedld.so \
  nm_res_nobar=build/exp/d_nm_res_nobar/libweightedld.so nm_res_1dma_nobar=build/exp/d_nm_res_1dma_nobar/libweightedld.so \
  noepi_res=build/exp/d_noepi_res_alds/libweightedld.so noepi_res_1dma=build/exp/d_noepi_res_1dma/libweightedld.so || exit 1
echo done
