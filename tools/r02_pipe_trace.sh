#!/bin/bash
# Kernel trace of the rehearsed N>1 pipeline at rank 0's 1/8 shard of C4,
# overlapped and device-serialised.  -> gpurun_out/TAG/
out=gpurun_out/${1:-r02pt}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $out/ovl -o ovl -- \
  python3 bench.py --rehearse-dist --rehearse-shard 8 --steps 100 --warmup 10 --no-cpu-baseline > $out/ovl.log 2>&1 || { echo "rocprof ovl failed $?"; exit 1; }
WLD_PIPE_SERIALIZE=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $out/ser -o ser -- \
  python3 bench.py --rehearse-dist --rehearse-shard 8 --steps 100 --warmup 10 --no-cpu-baseline > $out/ser.log 2>&1 || { echo "rocprof ser failed $?"; exit 1; }
echo done
