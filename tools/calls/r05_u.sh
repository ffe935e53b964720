#!/bin/bash
# round-5 GPU call U: raw wave timeline of the C2 item kernel (default build
# with stamps) for offline analysis
out=gpurun_out/r05u; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 200 $out/item_trace.log python3 tools/item_trace.py build/exp/i_trace/libweightedld.so c2 20 $out/item_trace_c2.npy || exit 1
echo done
