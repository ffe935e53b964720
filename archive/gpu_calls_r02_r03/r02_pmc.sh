#!/bin/bash
# Counter passes over the non-pipelined C4 bench (screen kernel + candidates),
# plus the screen/4-plane GPU tests.  -> gpurun_out/TAG/
tag=${1:-r02p}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
tools/gpu_step.sh 300 $out/screen_tests.txt python -u -m pytest tests/test_gpu_screen.py -q -s --timeout 300 --timeout-method thread || exit $?
tools/pmc_passes.sh --no-pipeline --steps 10 --warmup 3 --no-cpu-baseline || exit $?
rm -rf $out/pmc; mv gpurun_out/pmc $out/pmc; mv gpurun_out/pmc_*.log $out/
python3 tools/pmc_summary.py $out/pmc > $out/pmc_summary.txt
echo done
