#!/usr/bin/env python3
"""First pass of a fresh context against its steady state: the
wall time of the first wld_run after a load (it includes fp6_prepare and the
fp6 screen's sample run) and of later runs, on C4-size data.
    python tools/first_pass.py [random|ldblocks] [thr]"""
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402,F401

import bench  # noqa: E402
import weightedld_amd as W  # noqa: E402

data = sys.argv[1] if len(sys.argv) > 1 else "ldblocks"
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 0.05
N, L = 2000, 20000
buf = bench.synth(L, N) if data == "random" else bench.ld_blocks(L, N)
w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
warm = W.Context(0)  # HIP start-up and the first kernel loads, outside the timing
warm.load(buf, w)
warm.run(thr)
warm.close()
out = {"data": data, "thr": thr}
for rep in range(3):
    c = W.Context(0)
    c.load(buf, w)
    t0 = time.perf_counter()
    rows = c.run(thr)
    first = (time.perf_counter() - t0) * 1e3
    st = c.stats()
    info = {k: st[k] for k in ("screened", "screen_fp6", "fp6_sampled", "candidate_tiles", "pair_kernel_ms")}
    ts = []
    for _ in range(10):
        t0 = time.perf_counter()
        c.run(thr)
        ts.append((time.perf_counter() - t0) * 1e3)
    steady = statistics.median(ts)
    out["rep%d" % rep] = {"first_ms": first, "steady_ms": steady, "ratio": first / steady, "rows": rows,
                          "first_pass": info, "steady_pass": {k: c.stats()[k] for k in info}}
    c.close()
print(json.dumps(out))
