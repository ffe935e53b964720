#!/usr/bin/env python3
"""Writes bench.py's seeded synthetic alignment (bench_weighted_pair_ld.rs
distribution) as FASTA, one sequence per line with a trailing newline
(SURVEY App. A.1), for end-to-end CLI runs.
    tools/make_fasta.py N L out.fasta"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

N, L, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
codes = bench.synth(L, N)  # [L, N]
lut = np.frombuffer(b"ACGT-N", dtype=np.uint8)
with open(out, "wb") as f:
    for k in range(N):
        f.write(b">s%d\n" % k)
        f.write(lut[codes[:, k]].tobytes() + b"\n")
