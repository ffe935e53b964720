#!/bin/bash
# N>1 step pipeline A/B through an RCCL group of one: depth 2/3; kernels
# overlapped (ovl), device-serialised on the whole previous step (ser) or on its
# pair kernel only (pair, wld_run_after); rank 0's shard of an 8-way split (the
# per-rank work at N=8) and the whole C4.  -> gpurun_out/TAG/
out=gpurun_out/${1:-r02pa}; mkdir -p $out
export TMPDIR=/tmp
tools/gpu_step.sh 300 $out/pipe_tests.txt python -u -m pytest tests/test_gpu_parity.py -k pipelined -v --timeout 200 --timeout-method thread || exit $?
for rep in 1 2 3; do
for sh in 8 0; do
  [ $sh = 0 ] && [ $rep = 3 ] && continue
  for m in ovl:2 ser:2 pair:2 pair:3; do
    mode=${m%:*}; d=${m#*:}
    env=""; [ $mode = ser ] && env=1; [ $mode = pair ] && env=pair
    WLD_PIPE_SERIALIZE=$env tools/gpu_step.sh 200 $out/${mode}_d${d}_s${sh}_$rep.log python bench.py --rehearse-dist --rehearse-shard $sh --pipe-depth $d --no-cpu-baseline || exit $?
  done
done
done
echo done
