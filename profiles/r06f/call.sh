#!/bin/bash
# round-6 GPU call F: counters of the C4 fp6 screen before (round-5 library,
# built from a22dc03) and after (in-tree), two passes each; the traffic passes
# of the default C4 line and of the LD-block line (profiles/traffic.json)
out=gpurun_out/r06f; mkdir -p $out; export TMPDIR=/tmp
P2="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_INST_LDS"
for b in r05=build/exp/r05/libweightedld.so cur=weightedld_amd/libweightedld.so; do
  n=${b%%=*}; l=${b#*=}
  tools/gpu_step.sh 120 $out/pmcb_${n}_a.txt tools/pmc_build.sh ${n}_a $l c4 || exit $?
  PMC="$P2" tools/gpu_step.sh 120 $out/pmcb_${n}_b.txt tools/pmc_build.sh ${n}_b $l c4 || exit $?
done
tools/gpu_step.sh 400 $out/pmc_c4.txt tools/pmc_passes.sh --steps 5 --warmup 2 --settle-s 0 --no-cpu-baseline || exit $?
mv gpurun_out/pmc gpurun_out/r06f/pmc_c4; mv gpurun_out/pmc_*.log $out/ 2>/dev/null
tools/gpu_step.sh 400 $out/pmc_ldb.txt tools/pmc_passes.sh --steps 5 --warmup 2 --settle-s 0 --no-cpu-baseline --data ldblocks || exit $?
mv gpurun_out/pmc gpurun_out/r06f/pmc_ldb
echo done
