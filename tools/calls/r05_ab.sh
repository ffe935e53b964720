#!/bin/bash
# round-5 GPU call AB: kernel timeline of the rehearsed 1/8 shard (N>1 step
# path, three contexts in flight): gaps between screens
out=gpurun_out/r05ab; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/trace_shard8 -o s8 -- \
  python3 bench.py --rehearse-dist --rehearse-shard 8 --steps 200 --warmup 20 --no-cpu-baseline > $out/trace_shard8.log 2>&1 || { echo "trace failed"; exit 1; }
echo done
