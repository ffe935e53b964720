#!/usr/bin/env python3
"""Times the fp6 screen's give-up at C4-size linkage blocks: the first pass of
a fresh context (auto: fp6, given up, re-run on i8), the same forced on fp6
(no give-up), and on i8 alone; pair-kernel time from the context's stats.
    python tools/fp6_abandon_timing.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import weightedld_amd as W  # noqa: E402

buf = bench.ld_blocks(20000, 2000)
w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
for name, opt in (("auto", 1), ("forced", 2), ("i8", 0), ("auto", 1)):
    c = W.Context(0)
    c.set_option("screen_fp6", opt)
    c.load(buf, w)
    t = time.perf_counter()
    n = c.run(0.05)
    dt = (time.perf_counter() - t) * 1e3
    st = c.stats()
    t2 = time.perf_counter()
    c.run(0.05)
    dt2 = (time.perf_counter() - t2) * 1e3
    print("%-6s first run %.3f ms (pair %.3f, screen %.3f, screen_fp6 %d, cand %d, rows %d); second %.3f ms "
          "(screen_fp6 %d)" % (name, dt, st["pair_kernel_ms"], st["screen_ms"], st["screen_fp6"],
                               st["candidate_tiles"], n, dt2, c.stats()["screen_fp6"]), flush=True)
    c.close()
