#!/usr/bin/env python3
"""Row hand-over rates on one device (the in-process group's gather):
LD-block C4 data at thr 0.05 (~0.7 M rows of 20 bytes), then the median time of
  host      wld_rows_copy into pageable numpy arrays (what run_host_group does)
  pinned    wld_rows_copy into pinned host tensors
  device    wld_rows_copy_device into device tensors (HBM to HBM)
over 7 repetitions each; prints one JSON line."""
import ctypes
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import weightedld_amd as W  # noqa: E402
from weightedld_amd.api import _p  # noqa: E402
from weightedld_amd._lib import check, lib  # noqa: E402


def timed(fn, reps=7):
    t = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        t.append((time.perf_counter() - t0) * 1e3)
    return statistics.median(t)


def main():
    N, Ls, thr, _ = bench.CONFIGS["c4"]
    buf = bench.ld_blocks(Ls, N)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    ctx = W.Context(0, W.KERNEL_MFMA)
    ctx.load(buf, w)
    n = ctx.run(thr)
    nbytes = 20 * n
    h = [np.zeros(n, dtype=np.uint32), np.zeros(n, dtype=np.uint32)] + [np.zeros(n, dtype=np.float32) for _ in range(3)]
    cts = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_float, ctypes.c_float, ctypes.c_float]

    def host():
        check(lib().wld_rows_copy(ctx._h, *[_p(a, c) for a, c in zip(h, cts)]), "wld_rows_copy")

    pin = [torch.empty(n, dtype=torch.int32, pin_memory=True) for _ in range(5)]

    def pinned():
        check(lib().wld_rows_copy(ctx._h, *[ctypes.cast(t.data_ptr(), ctypes.POINTER(c)) for t, c in zip(pin, cts)]),
                "wld_rows_copy")

    dev = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(5)]

    def device():
        ctx.rows_copy_device(*[t.data_ptr() for t in dev])

    out = {"rows": n, "bytes": nbytes}
    for name, fn in (("host", host), ("pinned", pinned), ("device", device)):
        ms = timed(fn)
        out[name + "_ms"] = round(ms, 4)
        out[name + "_GBps"] = round(nbytes / ms / 1e6, 1)
    ref = ctx.rows()
    out["host_rows_equal_device"] = bool(np.array_equal(ref.site_a, dev[0].cpu().numpy().view(np.uint32)))
    ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
