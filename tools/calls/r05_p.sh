#!/bin/bash
# round-5 GPU call P: where the C2 item kernel's time goes (diagnostic builds,
# timing only): no compaction/stores; no epilogue; four workgroups per CU
out=gpurun_out/r05p; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 400 $out/ab_c2.log python3 tools/ab_builds.py --config c2 --reps 20 --rounds 3 \
  base=weightedld_amd/libweightedld.so nocomp=build/exp/i_nocomp/libweightedld.so \
  noepi=build/exp/i_noepi/libweightedld.so wg4=build/exp/i_wg4/libweightedld.so || exit 1
echo done
