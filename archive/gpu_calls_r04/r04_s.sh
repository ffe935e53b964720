#!/bin/bash
# round-4 GPU call S: the screens' bound on packed f32 (spk build) at C4
# (fp6 screen) and on LD blocks (i8 screen), with the persistent i8 screen
# (i8pipe build); then the fp6/screen/parity tests on the spk build
out=gpurun_out/r04s; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 400 $out/ab_c4.txt python tools/ab_builds.py --config c4 --reps 15 --rounds 3 \
  base=weightedld_amd/libweightedld.so spk=build/exp/spk/libweightedld.so || exit $?
WLD_AB_DATA=ldblocks WLD_AB_OPTS=screen_fp6=0 tools/gpu_step.sh 400 $out/ab_ld.txt python tools/ab_builds.py --config c4 --reps 15 --rounds 2 \
  base=weightedld_amd/libweightedld.so spk=build/exp/spk/libweightedld.so i8pipe=build/exp/i8pipe/libweightedld.so || exit $?
cp build/exp/spk/libweightedld.so weightedld_amd/libweightedld.so
tools/gpu_step.sh 600 $out/tests_spk.log python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fp6.py tests/test_gpu_screen.py tests/test_gpu_parity.py || exit $?
echo done
