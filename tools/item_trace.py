#!/usr/bin/env python3
"""Timeline of the full-run item kernel (ref_item_kernel<false>) from a
WLD_ITEM_TRACE build (tools/build_variant.sh; SRC=pair_valu, -DWLD_ITEM_TRACE=1):
per wave {HW_ID | XCC_ID << 32, start, sums done, end} of the last launch, in
wall_clock64 ticks (100 MHz = 10 ns).  Prints the launch span, the phases per
wave (sums, epilogue + compaction + scan ticket), the start/end spread, how
many workgroups each CU ran, and the busy fraction of each SIMD over the span.
    python tools/item_trace.py LIB.so [config=c2] [reps=20] [RAW.npy]"""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402,F401

import weightedld_amd._lib as L  # noqa: E402

L.LIB_PATH = os.path.abspath(sys.argv[1])
import bench  # noqa: E402
import weightedld_amd as W  # noqa: E402

config = sys.argv[2] if len(sys.argv) > 2 else "c2"
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
N, Ls, thr, _ = bench.CONFIGS[config]
buf = bench.synth(Ls, N)
w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
ctx = W.Context(0, W.KERNEL_MFMA)
ctx.load(buf, w)
lib = W.lib()
lib.wld_diag_item_trace.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_size_t, ctypes.c_int]
ms = []
for _ in range(reps):
    ctx.run(thr)
    ms.append(ctx.stats()["pair_kernel_ms"])
n_words = 65536 * 4
lib.wld_diag_item_trace(None, 0, 1)
ctx.run(thr)  # the traced launch
kms = ctx.stats()["pair_kernel_ms"]
out = (ctypes.c_ulonglong * n_words)()
assert lib.wld_diag_item_trace(out, n_words, 0) == 0
a = np.frombuffer(out, dtype=np.uint64).reshape(-1, 4)
a = a[a[:, 3] != 0]
if len(sys.argv) > 4:  # the raw records, for offline analysis
    np.save(sys.argv[4], a)
hw, t0, t1, t2 = a[:, 0], a[:, 1].astype(np.int64), a[:, 2].astype(np.int64), a[:, 3].astype(np.int64)
base = t0.min()
t0, t1, t2 = t0 - base, t1 - base, t2 - base
tick_us = 0.01
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
se = (hw >> 13) & 7
xcc = (hw >> 32) & 15
cu_id = (xcc * 8 + se) * 16 + cu
simd_id = cu_id * 4 + simd
span = t2.max()
res = {"config": config, "median_kernel_ms_untraced_runs": float(np.median(ms)), "traced_kernel_ms": kms,
       "waves": int(len(a)), "span_us": float(span * tick_us),
       "sums_us": {"p10": float(np.percentile(t1 - t0, 10) * tick_us), "median": float(np.median(t1 - t0) * tick_us),
                   "p90": float(np.percentile(t1 - t0, 90) * tick_us)},
       "epilogue_to_end_us": {"p10": float(np.percentile(t2 - t1, 10) * tick_us),
                              "median": float(np.median(t2 - t1) * tick_us),
                              "p90": float(np.percentile(t2 - t1, 90) * tick_us)},
       "start_us": {"p50": float(np.median(t0) * tick_us), "max": float(t0.max() * tick_us)},
       "end_us": {"min": float(t2.min() * tick_us), "p50": float(np.median(t2) * tick_us)}}
# workgroups per CU (wave 0 of each workgroup: 4 waves per workgroup)
wg_cu = cu_id[::4] if len(cu_id) % 4 == 0 else cu_id
u, c = np.unique(wg_cu, return_counts=True)
res["cus"] = int(len(u))
res["workgroups_per_cu"] = {str(k): int(v) for k, v in zip(*np.unique(c, return_counts=True))}
# per SIMD: time with at least one wave in its sums phase, over the span
busy_sums, busy_any = [], []
for s in np.unique(simd_id):
    m = simd_id == s
    for which, lst in ((t1, busy_sums), (t2, busy_any)):
        iv = sorted(zip(t0[m], which[m]))
        tot, cur_s, cur_e = 0, None, None
        for s0, e0 in iv:
            if cur_e is None or s0 > cur_e:
                if cur_e is not None:
                    tot += cur_e - cur_s
                cur_s, cur_e = s0, e0
            else:
                cur_e = max(cur_e, e0)
        tot += cur_e - cur_s
        lst.append(tot / span)
res["simd_frac_with_a_wave_in_sums"] = {"p10": float(np.percentile(busy_sums, 10)),
                                        "median": float(np.median(busy_sums)),
                                        "p90": float(np.percentile(busy_sums, 90))}
res["simd_frac_with_any_wave"] = {"median": float(np.median(busy_any))}
# waves per SIMD over the launch
per_simd = np.unique(simd_id, return_counts=True)[1]
res["waves_per_simd"] = {str(k): int(v) for k, v in zip(*np.unique(per_simd, return_counts=True))}
# active waves in their sums phase over time (20 bins)
bins = np.linspace(0, span, 21)
act = [int(((t0 <= b) & (t1 > b)).sum()) for b in bins[:-1]]
res["waves_in_sums_over_time"] = act
print(json.dumps(res))
