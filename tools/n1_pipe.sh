#!/bin/bash
# N=1 bench: pipelined over two contexts (default) vs --no-pipeline, interleaved
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
out=gpurun_out/n1p; mkdir -p $out
for r in 1 2 3; do
  for v in pipe nopipe; do
    a=""; [ $v = nopipe ] && a="--no-pipeline"
    for c in c4 c2; do
      timeout -k 10 200 python bench.py --no-cpu-baseline --config $c $a > $out/${v}_${c}_$r.log 2>&1 || { echo "bench $v $c failed"; tail -5 $out/${v}_${c}_$r.log; exit 1; }
      echo "$v $c $r $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*\|"rows_passing": [0-9]*' $out/${v}_${c}_$r.log | tr '\n' ' ')" | tee -a $out/summary.txt
    done
  done
done
