#!/bin/bash
# One SQ counter pass per build over the A/B child (C4, default kernel): tools/r02_pmc_variant.sh TAG VARIANT...
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for v in base "$@"; do
  lib=build/exp/$v/libweightedld.so; [ $v = base ] && lib=weightedld_amd/libweightedld.so
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE \
    --output-format csv -d $out/pmc_$v -o sq -- python3 tools/ab_builds.py --child $lib --config c4 --reps 5 > $out/pmc_$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
done
echo done
