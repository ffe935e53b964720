#!/bin/bash
# round-6 GPU call N: the candidate item loop's occupancy (no per-stage
# prefetch, 4/5/6 workgroups per CU) and A operands shared through LDS for
# items in one row block (as4/as5/as6), A/B on LD blocks at C4 size; the
# candidate tests on the as6 and nopf6 builds; the headline command under
# rocprofv3 with the pair kernels queued (no overlapping launches)
out=gpurun_out/r06n; mkdir -p $out; export TMPDIR=/tmp
B="base=weightedld_amd/libweightedld.so"
for v in nopf4 nopf5 nopf6 as4 as5 as6; do B="$B $v=build/exp/$v/libweightedld.so"; done
WLD_AB_DATA=ldblocks tools/gpu_step.sh 400 $out/ab_ldb.log python tools/ab_builds.py --config c4 --reps 20 --rounds 3 $B || exit $?
for v in as6 nopf6; do
  WLD_LIB_PATH=build/exp/$v/libweightedld.so tools/gpu_step.sh 300 $out/tests_$v.log python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_refsums.py tests/test_gpu_screen.py tests/test_gpu_i8pairs.py -m gpu || exit $?
done
WLD_PIPE_SERIALIZE=pair tools/gpu_step.sh 300 $out/prof_c4.log rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c4 -o c4 -- python3 bench.py --no-cpu-baseline || exit $?
echo done
