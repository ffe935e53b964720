#!/bin/bash
# GPU tests on the default build, then one-plane A/B against build/exp/kg8
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
out=gpurun_out/kg; mkdir -p $out
tools/gpu_step.sh 400 $out/tests.txt python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
B="base=weightedld_amd/libweightedld.so kg8=build/exp/kg8/libweightedld.so"
tools/gpu_step.sh 300 $out/ab_c4u.txt python -u tools/ab_builds.py --config c4 --unweighted --rounds 3 --reps 10 $B || exit $?
tools/gpu_step.sh 300 $out/ab_c5u.txt python -u tools/ab_builds.py --config c5 --unweighted --rounds 2 --reps 4 $B || exit $?
tools/gpu_step.sh 300 $out/ab_c4.txt python -u tools/ab_builds.py --config c4 --rounds 2 --reps 10 $B || exit $?
echo done
