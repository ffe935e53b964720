#!/bin/bash
# One GPU call: GPU tests against each experimental build, then interleaved A/B
# timing against the default build.
#   tools/ab_call.sh TAG CONFIGS NAME...   (builds under build/exp/NAME)
tag=$1; configs=$2; shift 2
out=gpurun_out/ab_$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
builds="base=weightedld_amd/libweightedld.so"
for n in "$@"; do
  [ -f build/exp/$n/DIAG ] || \
  WLD_LIB=build/exp/$n/libweightedld.so tools/gpu_step.sh 300 $out/tests_$n.txt \
    python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
  builds="$builds $n=build/exp/$n/libweightedld.so"
done
for c in $configs; do
  reps=10; [ "$c" = c5 ] && reps=4
  tools/gpu_step.sh 400 $out/ab_$c.txt python -u tools/ab_builds.py --config $c --rounds 3 --reps $reps $builds || exit $?
done
echo done
