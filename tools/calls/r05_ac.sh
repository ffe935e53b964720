#!/bin/bash
# round-5 GPU call AC: f32 16x16x4 MFMA issue rate by waves per SIMD and
# instruction pattern (tools/probes/f32_mfma_rate_probe.hip)
out=gpurun_out/r05ac; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 120 $out/f32_rate.log tools/probes/f32_mfma_rate_probe || exit $?
echo done
