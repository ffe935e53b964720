#!/bin/bash
# End-to-end CLI timing (main.rs-style logs) on synthetic FASTA:
#   tools/cli_e2e.sh -> gpurun_out/cli_e2e/*.log
out=gpurun_out/cli_e2e; mkdir -p $out
python3 tools/make_fasta.py 500 2000 /tmp/c2.fasta && python3 tools/make_fasta.py 2000 20000 /tmp/c4.fasta || exit 1
export RUST_LOG=debug
timeout -k 10 300 weightedld_amd/bin/weighted_ld --fasta-input /tmp/c2.fasta --pair-output /tmp/c2.tsv --r2-threshold 0.0 > $out/c2.log 2>&1 || exit $?
wc -l /tmp/c2.tsv >> $out/c2.log
timeout -k 10 300 weightedld_amd/bin/weighted_ld --fasta-input /tmp/c4.fasta --pair-output /tmp/c4.tsv --r2-threshold 0.05 > $out/c4.log 2>&1 || exit $?
wc -l /tmp/c4.tsv >> $out/c4.log
timeout -k 10 300 weightedld_amd/bin/weighted_ld --fasta-input /tmp/c4.fasta --pair-output /tmp/c4b.tsv --r2-threshold 0.001 > $out/c4_thr0001.log 2>&1 || exit $?
wc -l /tmp/c4b.tsv >> $out/c4_thr0001.log
timeout -k 10 300 weightedld_amd/bin/weighted_ld --fasta-input /tmp/c2.fasta --pair-output /tmp/c2g.tsv --r2-threshold 0.0 --gpu-prepass > $out/c2_gpu_prepass.log 2>&1 || exit $?
cmp /tmp/c2.tsv /tmp/c2g.tsv >> $out/c2_gpu_prepass.log 2>&1 && echo "identical to host-prepass TSV" >> $out/c2_gpu_prepass.log
