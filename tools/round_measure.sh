#!/bin/bash
# One GPU call: tests, bench lines, rocprofv3 kernel trace/stats, PMC passes.
#   tools/round_measure.sh TAG   -> gpurun_out/m_TAG/...
tag=${1:-r01}
out=gpurun_out/m_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 500 $out/gpu_tests.txt python -m pytest tests -m gpu -q || exit $?
tools/gpu_step.sh 300 $out/bench_c4_mfma.log python bench.py || exit $?
tools/gpu_step.sh 300 $out/bench_c4_valu.log python bench.py --kernel valu --steps 5 --warmup 1 --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $out/bench_c2.log python bench.py --config c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $out/bench_c4_unweighted.log python bench.py --unweighted --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $out/bench_c5.log python bench.py --config c5 --steps 5 --warmup 3 --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $out/bench_c4_rehearse.log python bench.py --rehearse-dist --no-cpu-baseline || exit $?
timeout -k 10 600 tools/cli_e2e.sh > $out/cli_e2e.log 2>&1 || { echo "cli_e2e failed $?"; exit 1; }
cp -r gpurun_out/cli_e2e $out/
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o c4 -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $out/prof.log 2>&1 || { echo "rocprof failed $?"; exit 1; }
for pass in "sq:SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
            "fetch:FETCH_SIZE GRBM_GUI_ACTIVE" "write:WRITE_SIZE GRBM_GUI_ACTIVE" "l2:TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  name=${pass%%:*}; ctrs=${pass#*:}
  timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d $out/pmc/$name -o $name -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $out/pmc_$name.log 2>&1 || { echo "pmc $name failed"; exit 1; }
done
echo done
