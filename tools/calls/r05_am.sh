#!/bin/bash
# round-5 GPU call AM: resident waves per CU of the producer/consumer fp6
# screen (nine-wave workgroups) against the default, by SQ_WAVE_CYCLES over
# GRBM_GUI_ACTIVE, C4 bench steps
out=gpurun_out/r05am; mkdir -p $out; cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
bargs="--steps 5 --warmup 2 --settle-s 0 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv \
  -d $out/base -o base -- python3 bench.py $bargs > $out/base.log 2>&1 || { echo "base pmc failed"; exit 1; }
WLD_LIB_PATH=build/exp/pc/libweightedld.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES \
  SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d $out/pc -o pc -- python3 bench.py $bargs > $out/pc.log 2>&1 \
  || { echo "pc pmc failed"; exit 1; }
echo done
