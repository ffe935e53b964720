"""Fixed per-call cost of wld_run_chunks: wall time of runs over 1 chunk and
over an 8-rank C4 shard, against their HIP-event kernel time.
    python tools/run_overhead.py"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import weightedld_amd as W  # noqa: E402

N, L, thr, _ = bench.CONFIGS["c4"]
buf = bench.synth(L, N)
w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
ctx = W.Context(0)
ctx.load(buf, w)
for name, (b, e) in (("1 chunk", (0, 1)), ("8-rank shard 0", ctx.shard_chunks(L, 8, 0)),
                     ("8-rank shard 7", ctx.shard_chunks(L, 8, 7)), ("full", (0, 0))):
    for _ in range(5):
        ctx.run_chunks(thr, b, e)
    wall, kern, order = [], [], []
    for _ in range(30):
        t0 = time.perf_counter()
        ctx.run_chunks(thr, b, e)
        wall.append((time.perf_counter() - t0) * 1e3)
        st = ctx.stats()
        kern.append(st["pair_kernel_ms"])
        order.append(st["order_ms"])
    print("%-16s wall %.3f ms  kernel %.3f ms  order %.3f ms  overhead %.3f ms" %
          (name, np.median(wall), np.median(kern), np.median(order),
           np.median(wall) - np.median(kern) - np.median(order)), flush=True)
