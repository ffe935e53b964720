#!/bin/bash
# round-5 GPU call AS: the wide-wave screen's epilogue share (timing build
# WLD_F6_DIAG 1: one compare instead of the bound; rows not meaningful) at C4, C5
out=gpurun_out/r05as; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 300 $out/ab_c4.log python3 tools/ab_builds.py --config c4 --reps 10 --rounds 3 \
  wide=weightedld_amd/libweightedld.so noepi=build/exp/noepi/libweightedld.so || exit 1
tools/gpu_step.sh 300 $out/ab_c5.log python3 tools/ab_builds.py --config c5 --reps 4 --rounds 2 \
  wide=weightedld_amd/libweightedld.so noepi=build/exp/noepi/libweightedld.so || exit 1
echo done
