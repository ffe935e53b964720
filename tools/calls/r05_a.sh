#!/bin/bash
# round-5 GPU call A: the fp6/bf6 dual-reading probe; baseline C4 bench on this box
out=gpurun_out/r05a; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 60 $out/probe.log tools/probes/fp6_dual_probe || exit 1
tools/gpu_step.sh 300 $out/bench_c4.log python3 bench.py --steps 20 --warmup 5 || exit 1
echo done
