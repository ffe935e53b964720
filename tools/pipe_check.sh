#!/bin/bash
# GPU tests, then bench's N>1 step path rehearsed at N=1 (RCCL group of one):
# pipelined vs one step at a time, C4 (no rows) and C2 at thr 0 (every pair a row)
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pipe; mkdir -p $out
tools/gpu_step.sh 400 $out/tests.txt python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread || exit $?
for a in "" "--no-pipeline"; do
  for c in c4 c2; do
    timeout -k 10 200 python bench.py --rehearse-dist --no-cpu-baseline --config $c $a > $out/rh_${c}${a}.log 2>&1 || { echo "bench $c $a failed"; tail -20 $out/rh_${c}${a}.log; exit 1; }
    echo "$c $a $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*\|"rows_passing": [0-9]*\|"parallelism": "[^"]*"' $out/rh_${c}${a}.log | tr '\n' ' ')" | tee -a $out/summary.txt
  done
done
timeout -k 10 200 python bench.py --no-cpu-baseline > $out/n1.log 2>&1 || exit 1
echo "n1 $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*' $out/n1.log | tr '\n' ' ')" | tee -a $out/summary.txt
