#!/bin/bash
# round-3 GPU call AR: XCD super-block size of the screen's launch order
# (capi.hip xcd_order kS: 8 shipped; 6, 11, 16 as -DWLD_XCD_SB builds):
# interleaved pair-kernel A/B at C4, then FETCH_SIZE per screen launch for 8 and 16
out=gpurun_out/r03ar; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python tools/ab_builds.py --config c4 --rounds 3 --reps 10 main=weightedld_amd/libweightedld.so \
  sb6=build/exp/sb6/libweightedld.so sb11=build/exp/sb11/libweightedld.so sb16=build/exp/sb16/libweightedld.so \
  > $out/ab.txt 2>&1 || { echo "ab failed $?"; exit 1; }
cat $out/ab.txt | tail -8
cp weightedld_amd/libweightedld.so /tmp/lib_main.so
for v in main sb16; do
if [ $v = main ]; then cp /tmp/lib_main.so weightedld_amd/libweightedld.so; else cp build/exp/$v/libweightedld.so weightedld_amd/libweightedld.so; fi
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_$v -o fetch -- \
  python3 bench.py --no-pipeline --steps 10 --warmup 2 --settle-s 0 --no-cpu-baseline > $out/pmc_$v.log 2>&1 || { echo "pmc failed $?"; cp /tmp/lib_main.so weightedld_amd/libweightedld.so; exit 1; }
done
cp /tmp/lib_main.so weightedld_amd/libweightedld.so
echo done
