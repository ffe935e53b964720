#!/bin/bash
# round-5 GPU call Q: the candidate-entry guard test (WLD_OPT_TEST_GUARD) and
# the screen suite; then call P's C2 diagnostics
out=gpurun_out/r05q; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 600 $out/tests_screen.log python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_screen.py || exit 1
tools/calls/r05_p.sh || exit 1
# rank 0's 1/8 shard of C4: tile pairs vs single tiles
tools/gpu_step.sh 300 gpurun_out/r05q/ab_shard8.log env WLD_AB_SHARD=8 python3 tools/ab_builds.py --config c4 --reps 20 \
  --rounds 3 pairs=weightedld_amd/libweightedld.so single=build/exp/single_b4/libweightedld.so || exit 1
tools/gpu_step.sh 200 gpurun_out/r05q/item_trace.log python3 tools/item_trace.py build/exp/i_trace/libweightedld.so c2 20 || exit 1
echo done
