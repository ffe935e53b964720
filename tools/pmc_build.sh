#!/bin/bash
# Counter pass over one experimental build (tools/ab_builds.py child mode):
#   tools/pmc_build.sh NAME LIB [config]  -> gpurun_out/pmcb/NAME/
# PMC="counter ..." replaces the default counter set (one pass: at most 8 SQ_,
# 4 TCC_ counters; GRBM_GUI_ACTIVE gives the clock)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
name=$1; lib=$2; cfg=${3:-c4}
pmc=${PMC:-GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS}
timeout -k 10 300 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/pmcb/$name -o $name -- \
  python3 tools/ab_builds.py --child $lib --config $cfg --reps 3 > gpurun_out/pmcb_$name.log 2>&1
