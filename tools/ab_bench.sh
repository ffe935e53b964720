#!/bin/bash
# Interleaved bench.py wall-clock A/B of the default build against
# experimental builds (build/exp/NAME), same box:
#   tools/ab_bench.sh TAG "BENCH ARGS" NAME...   -> gpurun_out/abb_TAG/summary.txt
tag=$1; args=$2; shift 2
out=gpurun_out/abb_$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do
  for n in base "$@"; do
    lib=weightedld_amd/libweightedld.so; [ $n = base ] || lib=build/exp/$n/libweightedld.so
    WLD_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline $args > $out/${n}_$r.log 2>&1 || { echo "bench $n failed"; exit 1; }
    echo "$n $r $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*' $out/${n}_$r.log | tr '\n' ' ')" | tee -a $out/summary.txt
  done
done
