#!/usr/bin/env python3
"""Dense bitwise comparison of the persistent LDS kernel against the site-major
kernel (both exact-integer MFMA paths, identical epilogue), to localise
differences by tile / wave / row / column."""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402,F401

import weightedld_amd as W  # noqa: E402
from test_gpu_parity import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=4096)
    ap.add_argument("--N", type=int, default=2000)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--thr", type=float, default=0.001)
    a = ap.parse_args()
    buf = synth(a.L, a.N, 5)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    os.environ["WLD_MFMA_LAYOUT"] = "rows"
    ref = W.Context(0, W.KERNEL_MFMA)
    ref.load(buf, w)
    os.environ.pop("WLD_MFMA_LAYOUT")
    ctx = W.Context(0, W.KERNEL_MFMA)
    ctx.load(buf, w)
    rd = ref.dense(a.L)
    iu = np.triu_indices(a.L, 1)
    for run in range(a.runs):
        gd = ctx.dense(a.L)
        bad = np.zeros((a.L, a.L), dtype=bool)
        for k in range(3):
            x, y = gd[k].view(np.uint32), rd[k].view(np.uint32)
            bad |= x != y
        bad[np.tril_indices(a.L)] = False
        ia, ib = np.nonzero(bad)
        out = {"run": run, "mode": "dense", "bad": int(len(ia))}
        if len(ia):
            out["rows_mod32"] = np.bincount(ia % 32, minlength=32).tolist()
            out["cols_mod32"] = np.bincount(ib % 32, minlength=32).tolist()
            out["wave_rc"] = np.bincount(((ia % 64) // 32) * 2 + (ib % 64) // 32, minlength=4).tolist()
            out["n_tiles"] = len(set(zip((ia // 64).tolist(), (ib // 64).tolist())))
            out["sample"] = [(int(p), int(q), float(gd[2][p, q]), float(rd[2][p, q])) for p, q in zip(ia[:6], ib[:6])]
        print(json.dumps(out), flush=True)
    n_ref = ref.run(a.thr)
    for run in range(a.runs):
        n = ctx.run(a.thr)
        print(json.dumps({"run": run, "mode": "rows", "thr": a.thr, "n": n, "n_ref": n_ref}), flush=True)


if __name__ == "__main__":
    main()
