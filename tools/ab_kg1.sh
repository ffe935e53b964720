#!/bin/bash
# One-plane group-shape A/B: tests on each variant, then interleaved timing
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
out=gpurun_out/kg1; mkdir -p $out
for n in "$@"; do
  WLD_LIB=build/exp/$n/libweightedld.so tools/gpu_step.sh 300 $out/tests_$n.txt \
    python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "plane or unweighted or cli" || exit $?
done
B="base=weightedld_amd/libweightedld.so"; for n in "$@"; do B="$B $n=build/exp/$n/libweightedld.so"; done
tools/gpu_step.sh 300 $out/ab_c4u.txt python -u tools/ab_builds.py --config c4 --unweighted --rounds 3 --reps 10 $B || exit $?
tools/gpu_step.sh 300 $out/ab_c5u.txt python -u tools/ab_builds.py --config c5 --unweighted --rounds 2 --reps 4 $B || exit $?
echo done
