#!/bin/bash
# round-6 GPU call B: fp6 screen A/B at C4, C5 and the 1/8 shard: base (round-5
# kernel), cur (per-wave DMA bases), nt3 (tile triples, 6 waves, 2 WG/CU);
# then the fp6/screen tests on the in-tree library and on the nt3 build
out=gpurun_out/r06b; mkdir -p $out; export TMPDIR=/tmp
B="base=build/exp/base/libweightedld.so cur=weightedld_amd/libweightedld.so nt3=build/exp/nt3/libweightedld.so pk=build/exp/pk/libweightedld.so"
tools/gpu_step.sh 300 $out/ab_c4.log python tools/ab_builds.py --config c4 --reps 30 --rounds 3 $B || exit $?
tools/gpu_step.sh 300 $out/ab_c5.log python tools/ab_builds.py --config c5 --reps 6 --rounds 2 $B || exit $?
WLD_AB_SHARD=8 tools/gpu_step.sh 200 $out/ab_s8.log python tools/ab_builds.py --config c4 --reps 40 --rounds 3 $B || exit $?
tools/gpu_step.sh 400 $out/tests_cur.log python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fp6.py tests/test_gpu_screen.py -m gpu || exit $?
WLD_LIB_PATH=build/exp/nt3/libweightedld.so tools/gpu_step.sh 400 $out/tests_nt3.log python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fp6.py tests/test_gpu_screen.py -m gpu || exit $?

WLD_LIB_PATH=build/exp/pk/libweightedld.so tools/gpu_step.sh 400 $out/tests_pk.log python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fp6.py tests/test_gpu_screen.py -m gpu || exit $?
echo done
