#!/bin/bash
# round-3 GPU call AI: the pair phase's event marks (2, 6, 3) with a device-scope
# release (evdev) or no system fence (evnone) instead of the default
# system-scope fence (evsys): bench ms/step A/B (in-tree .so swapped) and a
# rocprofv3 kernel trace of each for the screen-to-screen gaps; then the GPU
# suite on the evdev build
out=gpurun_out/r03ai; mkdir -p $out; export TMPDIR=/tmp
for r in 1 2; do
  for b in evsys evdev evnone; do
    cp build/exp/$b/libweightedld.so weightedld_amd/libweightedld.so
    tools/gpu_step.sh 200 $out/bench_${b}_$r.log python bench.py --no-cpu-baseline || exit $?
  done
done
for b in evsys evdev evnone; do
  cp build/exp/$b/libweightedld.so weightedld_amd/libweightedld.so
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/prof_$b -o c4 -- \
    python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > $out/prof_$b.log 2>&1 || { echo "rocprof $b failed $?"; exit 1; }
done
cp build/exp/evdev/libweightedld.so weightedld_amd/libweightedld.so
tools/gpu_step.sh 900 $out/gpu_tests.txt python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread || exit $?
echo done
