#!/bin/bash
# round-5 GPU call Y: where a fresh context's first pass spends its time now
# (HIP API + kernel trace of tools/first_pass.py on random data)
out=gpurun_out/r05y; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $out/trace_first -o first -- \
  python3 tools/first_pass.py random 0.05 > $out/trace_first.log 2>&1 || { echo "trace failed"; exit 1; }
python3 tools/trace_timeline.py $out/trace_first 1 90 > $out/trace_first_timeline.txt
echo done
