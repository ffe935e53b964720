#!/bin/bash
# rehearsed N>1 path: kernels serialised by an event vs free to overlap the
# previous step's tail (WLD_PIPE_OVERLAP=1), interleaved
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
out=gpurun_out/povl; mkdir -p $out
for r in 1 2 3; do
  for v in ser ovl; do
    e=""; [ $v = ser ] && e="WLD_PIPE_SERIALIZE=1"
    env $e timeout -k 10 200 python bench.py --rehearse-dist --no-cpu-baseline $1 > $out/${v}_$r.log 2>&1 || { echo "bench $v failed"; exit 1; }
    echo "$v $r $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*' $out/${v}_$r.log | tr '\n' ' ')" | tee -a $out/summary.txt
  done
done
