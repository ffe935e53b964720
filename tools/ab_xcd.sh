cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
out=gpurun_out/xcd; mkdir -p $out
WLD_TILE_ORDER=xcd tools/gpu_step.sh 400 $out/tests_xcd.txt python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
B="base=weightedld_amd/libweightedld.so rows=weightedld_amd/libweightedld.so@WLD_TILE_ORDER=rows"
tools/gpu_step.sh 300 $out/ab_c4u.txt python -u tools/ab_builds.py --config c4 --unweighted --rounds 3 --reps 10 $B || exit $?
tools/gpu_step.sh 300 $out/ab_c4.txt python -u tools/ab_builds.py --config c4 --rounds 3 --reps 10 $B || exit $?
tools/gpu_step.sh 300 $out/ab_c5.txt python -u tools/ab_builds.py --config c5 --rounds 2 --reps 4 $B || exit $?
echo done
