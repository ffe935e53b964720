#!/bin/bash
# Counter passes (one rocprofv3 --pmc run each, kernel-trace only, no sys/runtime
# trace) over a short bench run; outputs under gpurun_out/pmc/<pass>/.
#   tools/pmc_passes.sh [bench args...]
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
args="$*"
[ -z "$args" ] && args="--steps 5 --warmup 2 --no-cpu-baseline"
run() {
  name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc/$name -o $name -- \
    python3 bench.py $args > gpurun_out/pmc_$name.log 2>&1
  rc=$?; echo "[pmc] $name rc=$rc"; return $rc
}
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE &&
run fetch FETCH_SIZE GRBM_GUI_ACTIVE &&
run write WRITE_SIZE GRBM_GUI_ACTIVE &&
run l2 TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE &&
run lds SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE
