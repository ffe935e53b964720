#!/usr/bin/env python3
"""Per-tile phase durations from a WLD_EXP_STAMPS build (wave 0 of each tile):
loop = start..loop end, epilogue = loop end..epilogue end (shader cycles)."""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402,F401

import weightedld_amd._lib as _L  # noqa: E402
_L.LIB_PATH = os.path.abspath(sys.argv[1])
import bench  # noqa: E402
import weightedld_amd as W  # noqa: E402

N, L, thr, _ = bench.CONFIGS["c4"]
buf = bench.synth(L, N)
w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
ctx = W.Context(0, W.KERNEL_MFMA)
ctx.load(buf, w)
ctx.run(thr)
ctx.run(thr)
ms = ctx.stats()["pair_kernel_ms"]
n = min(ctx.stats().get("tiles", 49141), 1 << 18)
n = 49141
arr = (ctypes.c_ulonglong * (3 * n))()
W.lib().wld_debug_stamps_copy(arr, n)
a = np.frombuffer(arr, dtype=np.uint64).reshape(n, 3).astype(np.int64)
loop = a[:, 1] - a[:, 0]
epi = a[:, 2] - a[:, 1]
span = a[:, 2].max() - a[:, 0].min()
print(json.dumps({"kernel_ms": ms, "span_cycles": int(span), "ghz_est": span / (ms * 1e6),
                  "loop_med": float(np.median(loop)), "loop_p90": float(np.percentile(loop, 90)),
                  "epi_med": float(np.median(epi)), "epi_p90": float(np.percentile(epi, 90)),
                  "tile_med": float(np.median(loop + epi))}))
