#!/bin/bash
# round-3 GPU call M: empty-slot fix (parity), then SQ/LDS counter passes of
# the LD-block bench (the screen, the reference-order candidate kernel and the
# full reference-order kernel of the unscreened leg)
out=gpurun_out/r03m; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 900 $out/tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_refsums.py tests/test_gpu_parity.py -k "not full" || exit $?
args="--data ldblocks --steps 5 --warmup 2 --settle-s 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $out/pmc_sq -o sq -- python3 bench.py $args > $out/pmc_sq.log 2>&1 || { echo "pmc sq failed $?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_lds -o lds -- python3 bench.py $args > $out/pmc_lds.log 2>&1 || { echo "pmc lds failed $?"; exit 1; }
echo done
