#!/bin/bash
# round-5 GPU call AK: dist / multi / bench / parity tests after trimming the
# per-step host calls; rehearsed 1/8 shard three times
out=gpurun_out/r05ak; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 700 $out/tests.log python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_dist.py tests/test_gpu_multi.py tests/test_gpu_parity.py tests/test_bench.py -m gpu || exit 1
for rep in 1 2 3; do
  tools/gpu_step.sh 200 $out/shard8_$rep.log python bench.py --rehearse-dist --rehearse-shard 8 --no-cpu-baseline || exit $?
done
echo done
