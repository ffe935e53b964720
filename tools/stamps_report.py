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
ctx.run(thr)  # the stamps of this (last) launch are reported
ms = ctx.stats()["pair_kernel_ms"]
n = min(ctx.stats().get("tiles", 49141), 1 << 18)
n = 49141
arr = (ctypes.c_ulonglong * (4 * n))()
W.lib().wld_debug_stamps_copy(arr, n)
a = np.frombuffer(arr, dtype=np.uint64).reshape(n, 4).astype(np.int64)
pro = a[:, 1] - a[:, 0]
loop = a[:, 2] - a[:, 1]
epi = a[:, 3] - a[:, 2]
span = a[:, 3].max() - a[:, 0].min()
# per-SIMD occupancy view: sum of wave-0 busy time over all tiles / (span * 2 WG slots * 256 CUs)
busy = float((a[:, 3] - a[:, 0]).sum()) / (span * 512.0)
print(json.dumps({"kernel_ms": ms, "span_units": int(span), "units_per_ns": span / (ms * 1e6),
                  "slot_occupancy": busy, "pro_med": float(np.median(pro)), "pro_p90": float(np.percentile(pro, 90)),
                  "loop_med": float(np.median(loop)), "loop_p90": float(np.percentile(loop, 90)),
                  "epi_med": float(np.median(epi)), "epi_p90": float(np.percentile(epi, 90)),
                  "tile_med": float(np.median(loop + epi))}))
