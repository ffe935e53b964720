#!/bin/bash
# FETCH/WRITE/L2 counter passes over the non-pipelined C4 bench (screen kernel) -> gpurun_out/TAG/pmc
tag=${1:-r02t}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
run() {
  name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $out/pmc/$name -o $name -- \
    python3 bench.py --no-pipeline --steps 10 --warmup 3 --no-cpu-baseline > $out/pmc_$name.log 2>&1
  rc=$?; echo "[pmc] $name rc=$rc"; return $rc
}
run fetch FETCH_SIZE GRBM_GUI_ACTIVE &&
run write WRITE_SIZE GRBM_GUI_ACTIVE &&
run l2 TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE &&
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE &&
echo done
