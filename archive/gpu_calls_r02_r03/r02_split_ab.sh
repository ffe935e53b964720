#!/bin/bash
# Split screen launch (full waves + partial last wave, hand-off event between):
# screen + pipeline GPU tests, then the rehearsed per-rank step (1/8 shard) and
# the N=1 C4 line.  -> gpurun_out/TAG/
out=gpurun_out/${1:-r02sa}; mkdir -p $out
export TMPDIR=/tmp
tools/gpu_step.sh 500 $out/tests.txt python -u -m pytest tests/test_gpu_screen.py tests/test_gpu_parity.py -k "screen or pipelined or race" -q --timeout 200 --timeout-method thread || exit $?
for rep in 1 2 3; do
  tools/gpu_step.sh 200 $out/s8_$rep.log python bench.py --rehearse-dist --rehearse-shard 8 --no-cpu-baseline || exit $?
  tools/gpu_step.sh 200 $out/s4_$rep.log python bench.py --rehearse-dist --rehearse-shard 4 --no-cpu-baseline || exit $?
done
tools/gpu_step.sh 200 $out/c4.log python bench.py --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/c4_rehearse.log python bench.py --rehearse-dist --no-cpu-baseline || exit $?
echo done
