#!/usr/bin/env python3
"""Per-tile phase durations from a WLD_EXP_STAMPS build (wave 0 of each tile):
prologue = start..first group, loop = first group..loop end, epilogue = loop
end..epilogue end (s_memtime units), plus the co-residency view: per CU
(XCC, SE, SH, CU from HW_ID/XCC_ID), the fraction of the time some tile is
resident during which NO resident tile is in its loop (matrix cores idle for
lack of a looping wave), and how often the two tiles of a CU overlap their
non-loop phases.
    python tools/stamps_report.py LIB [config]"""
import ctypes
import json
import os
import sys
from collections import defaultdict

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402,F401

import weightedld_amd._lib as _L  # noqa: E402
_L.LIB_PATH = os.path.abspath(sys.argv[1])
import bench  # noqa: E402
import weightedld_amd as W  # noqa: E402

cfg = sys.argv[2] if len(sys.argv) > 2 else "c4"
N, L, thr, _ = bench.CONFIGS[cfg]
buf = bench.synth(L, N)
w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
ctx = W.Context(0, W.KERNEL_MFMA)
ctx.load(buf, w)
for _ in range(6):
    ctx.run(thr)  # clocks up; the stamps of the last launch are reported
ms = ctx.stats()["pair_kernel_ms"]
T = (L + 63) // 64
n = min(T * (T + 1) // 2, 1 << 18)
K = 5
arr = (ctypes.c_ulonglong * (K * n))()
W.lib().wld_debug_stamps_copy(arr, n)
a = np.frombuffer(arr, dtype=np.uint64).reshape(n, K)
st = a[:, :4].astype(np.int64)
hw = (a[:, 4] & 0xFFFFFFFF).astype(np.int64)
xcc = (a[:, 4] >> 32).astype(np.int64) & 0xF
pro = st[:, 1] - st[:, 0]
loop = st[:, 2] - st[:, 1]
epi = st[:, 3] - st[:, 2]
cu = (hw >> 8) & 0xF
sh = (hw >> 12) & 1
se = (hw >> 13) & 0x7
simd = (hw >> 4) & 3
key = xcc * 1000 + se * 100 + sh * 20 + cu
out = {"config": cfg, "kernel_ms": ms, "tiles": int(n),
       "pro_med": float(np.median(pro)), "loop_med": float(np.median(loop)), "epi_med": float(np.median(epi)),
       "distinct_cus": int(len(np.unique(key))), "simd_of_wave0": np.bincount(simd, minlength=4).tolist()}
# per-CU timeline sweep: events +1/-1 for resident and for looping
idle, resident_t, pair_nonloop, pairs = 0, 0, 0, 0
groups = defaultdict(list)
for i in range(n):
    groups[int(key[i])].append(i)
for k, idx in groups.items():
    ev = []
    for i in idx:
        ev.append((st[i, 0], 1, 0))
        ev.append((st[i, 3], -1, 0))
        ev.append((st[i, 1], 0, 1))
        ev.append((st[i, 2], 0, -1))
    ev.sort()
    res = lp = 0
    last = ev[0][0]
    for t, dr, dl in ev:
        if res > 0:
            resident_t += t - last
            if lp == 0:
                idle += t - last
        res += dr
        lp += dl
        last = t
out["cu_time_no_tile_looping_frac"] = idle / max(resident_t, 1)
print(json.dumps(out))
