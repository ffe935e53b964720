#!/bin/bash
# rocprofv3 kernel traces: f32-MFMA fallback, one-plane kernel, and the
# rehearsed N>1 step path pipelined vs not (gaps between pair kernels)
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pex; mkdir -p $out
for v in "valu:--kernel valu --steps 5 --warmup 1" "unw:--unweighted --steps 20 --warmup 5" \
         "pipe:--rehearse-dist --steps 30 --warmup 5" "nopipe:--rehearse-dist --no-pipeline --steps 30 --warmup 5"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$n -o $n -- \
    python3 bench.py --no-cpu-baseline $a > $out/$n.log 2>&1 || { echo "prof $n failed"; exit 1; }
done
echo done
