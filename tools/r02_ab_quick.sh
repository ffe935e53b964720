#!/bin/bash
# A/B of experimental builds at C4 only (speed, no tests): tools/r02_ab_quick.sh TAG VARIANT...
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
builds="base=weightedld_amd/libweightedld.so"
for v in "$@"; do builds="$builds $v=build/exp/$v/libweightedld.so"; done
timeout -k 10 500 python -u tools/ab_builds.py --config c4 --reps ${REPS:-10} --rounds ${ROUNDS:-3} $builds > $out/ab_c4.txt 2>&1 || exit 1
echo done
