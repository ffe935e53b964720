#!/bin/bash
# (experiment: the -DWLD_EV_NOTIMING variant was not kept; DESIGN.md §6, "Between screens")
# round-3 GPU call AQ: do timestamp-free per-pass events (hipEventDisableTiming,
# build/exp/evnt = -DWLD_EV_NOTIMING on capi.hip) shorten the gaps between
# screens?  C4 default bench, the two libraries interleaved, three passes
out=gpurun_out/r03aq; mkdir -p $out; export TMPDIR=/tmp
cp weightedld_amd/libweightedld.so /tmp/lib_main.so
for pass in 1 2 3; do for v in main evnt; do
if [ $v = main ]; then cp /tmp/lib_main.so weightedld_amd/libweightedld.so; else cp build/exp/evnt/libweightedld.so weightedld_amd/libweightedld.so; fi
tools/gpu_step.sh 200 $out/p${pass}_c4_$v.log python bench.py --no-cpu-baseline || exit $?
done; done
cp build/exp/evnt/libweightedld.so weightedld_amd/libweightedld.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o c4_evnt -- \
  python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > $out/prof_c4.log 2>&1 || { echo "rocprof failed $?"; exit 1; }
cp /tmp/lib_main.so weightedld_amd/libweightedld.so
echo done
