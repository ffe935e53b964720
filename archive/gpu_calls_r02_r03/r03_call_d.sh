#!/bin/bash
# round-3 GPU call D: new tests (unweighted C3, multi-rank GPU steps), the f32
# reference kernel at 2 vs 3 workgroups per CU (A/B), LD-block and C4 lines
out=gpurun_out/r03d; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 700 $out/gpu_tests_new.txt python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_multi.py tests/test_gpu_parity.py tests/test_gpu_refsums.py -m gpu -v -rf --timeout 300 --timeout-method thread || exit $?
WLD_AB_DATA=ldblocks tools/gpu_step.sh 300 $out/ab_refwg_ldblocks.txt python tools/ab_builds.py --config c4 --reps 8 --rounds 3 wg2=build/exp/refwg2/libweightedld.so wg3=build/exp/refwg3/libweightedld.so || exit $?
tools/gpu_step.sh 300 $out/ab_refwg_c4_thr0.txt python tools/ab_builds.py --config c4 --thr 0.0 --reps 3 --rounds 2 wg2=build/exp/refwg2/libweightedld.so wg3=build/exp/refwg3/libweightedld.so || exit $?
tools/gpu_step.sh 300 $out/bench_c4_ldblocks.log python bench.py --data ldblocks --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $out/bench_c4_20_5.log python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
echo done
