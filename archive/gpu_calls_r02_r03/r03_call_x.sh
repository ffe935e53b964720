#!/bin/bash
# round-3 GPU call X: the committed tree's default bench (with the CPU
# baseline), its rocprofv3 kernel stats, and the PMC traffic passes of the
# non-pipelined C4 bench (screen kernel) for profiles/traffic.json
out=gpurun_out/r03x; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 400 $out/bench_c4.log python bench.py || exit $?
tools/gpu_step.sh 300 $out/bench_c4_20_5.log python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o c4 -- \
  python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > $out/prof_c4.log 2>&1 || { echo "rocprof failed $?"; exit 1; }
cd /tmp && cd "$GRAFT_REPO_ROOT"
run() {
  name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $out/pmc/$name -o $name -- \
    python3 bench.py --no-pipeline --steps 10 --warmup 3 --settle-s 0 --no-cpu-baseline > $out/pmc_$name.log 2>&1
  rc=$?; echo "[pmc] $name rc=$rc"; return $rc
}
run fetch FETCH_SIZE GRBM_GUI_ACTIVE &&
run write WRITE_SIZE GRBM_GUI_ACTIVE &&
run l2 TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE &&
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE &&
echo done
