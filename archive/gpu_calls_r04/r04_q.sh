#!/bin/bash
# round-4 GPU call Q: workgroup placement probe; the fp6 screen with the
# first round's workgroups of a CU started apart (stagger builds); then
# call R's steps (the pipelined fp6 screen)
out=gpurun_out/r04q; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 60 tools/probes/place_probe > $out/place.txt 2>&1 || { echo "probe failed"; exit 1; }
tools/gpu_step.sh 400 $out/ab_c4.txt python tools/ab_builds.py --config c4 --reps 15 --rounds 2 \
  base=weightedld_amd/libweightedld.so s8k=build/exp/stag8128/libweightedld.so s16k=build/exp/stag16256/libweightedld.so || exit $?
out=gpurun_out/r04r; mkdir -p $out
B="base=weightedld_amd/libweightedld.so pipe=build/exp/pipe/libweightedld.so pipesgb=build/exp/pipesgb/libweightedld.so pipepk=build/exp/pipepk/libweightedld.so"
tools/gpu_step.sh 560 $out/ab_c4.txt python tools/ab_builds.py --config c4 --reps 15 --rounds 2 $B || exit $?
tools/gpu_step.sh 200 $out/ab_c4_thr.txt python tools/ab_builds.py --config c4 --thr 0.02 --reps 3 --rounds 1 \
  base=weightedld_amd/libweightedld.so@WLD_AB_OPTS=screen_fp6=2 pipepk=build/exp/pipepk/libweightedld.so@WLD_AB_OPTS=screen_fp6=2 || exit $?
cp build/exp/pipepk/libweightedld.so weightedld_amd/libweightedld.so
tools/gpu_step.sh 600 $out/tests_pipepk.log python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fp6.py tests/test_gpu_screen.py tests/test_gpu_parity.py || exit $?
echo done
