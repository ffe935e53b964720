#!/bin/bash
# SQ counter passes on the C4 bench (pair kernels), wide and 64x64 screens. -> gpurun_out/TAG/
tag=${1:-r02p2}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
for v in ${VARIANTS:-"i8:" "fp4:--fp4-screen"}; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d $out/pmc_$n/sq -o sq -- python3 bench.py --no-pipeline --steps 10 --warmup 3 --no-cpu-baseline $a > $out/sq_$n.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM GRBM_GUI_ACTIVE \
    --output-format csv -d $out/pmc_$n/lds -o lds -- python3 bench.py --no-pipeline --steps 10 --warmup 3 --no-cpu-baseline $a > $out/lds_$n.log 2>&1 || exit 1
done
python3 tools/pmc_summary.py $out > $out/pmc_summary.txt
echo done
