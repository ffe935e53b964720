#!/bin/bash
# GPU tests, then the f32 fallback on the matrix cores vs the VALU loop
# (WLD_VALU_PLAIN=1), interleaved, bench.py --kernel valu at C4
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
out=gpurun_out/valu; mkdir -p $out
tools/gpu_step.sh 400 $out/tests.txt python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread || exit $?
for r in 1 2; do
  for v in mf plain; do
    env_=""; [ $v = plain ] && env_="WLD_VALU_PLAIN=1"
    env $env_ timeout -k 10 200 python bench.py --kernel valu --steps 10 --warmup 2 --no-cpu-baseline > $out/${v}_$r.log 2>&1 || { echo "bench $v failed"; exit 1; }
    echo "$v $r $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*\|"frac": [0-9.]*' $out/${v}_$r.log | head -3 | tr '\n' ' ')" | tee -a $out/summary.txt
  done
done
