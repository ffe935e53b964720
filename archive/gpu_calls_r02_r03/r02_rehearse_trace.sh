#!/bin/bash
# Kernel + copy trace of the rehearsed N>1 step path (RCCL group of one) at C4,
# against the plain pipelined loop: where the step's extra time goes.
out=gpurun_out/${1:-r02rt}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $out/reh -o reh -- \
  python3 bench.py --rehearse-dist --steps 40 --warmup 5 --no-cpu-baseline > $out/reh.log 2>&1 || { echo "rocprof reh failed $?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $out/plain -o plain -- \
  python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > $out/plain.log 2>&1 || { echo "rocprof plain failed $?"; exit 1; }
echo done
