#!/bin/bash
# round-6 GPU call O: the f32 32x32x2 quadrant-form probe (order of the two
# k products, rate at 1..8 waves per SIMD); the candidate tests on the as6
# build again, verbose, with a longer limit (call N's 300 s ran out after 56)
out=gpurun_out/r06o; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 120 $out/probe.log build/probes/f32_mfma32q_probe || exit $?
WLD_LIB_PATH=build/exp/as6/libweightedld.so tools/gpu_step.sh 700 $out/tests_as6.log python3 -u -m pytest -x -v --durations=15 --timeout 120 --timeout-method thread tests/test_gpu_refsums.py tests/test_gpu_screen.py tests/test_gpu_i8pairs.py -m gpu || exit $?
echo done
