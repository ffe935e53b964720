#!/usr/bin/env python3
"""Debug helper: run a pair-kernel variant repeatedly on a bench config and
check every emitted row against the CPU oracle (single pair, f32 reference
semantics) and the f64 value of the same sums."""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import torch  # noqa: E402,F401

import _oracle as O  # noqa: E402
import bench  # noqa: E402
import weightedld_amd as W  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--kernel", default="mfma")
    ap.add_argument("--runs", type=int, default=10)
    ap.add_argument("--thr", type=float, default=None)
    args = ap.parse_args()
    N, L, thr, _ = bench.CONFIGS[args.config]
    if args.thr is not None:
        thr = args.thr
    buf = bench.synth(L, N)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    ctx = W.Context(0, W.KERNEL_MFMA if args.kernel == "mfma" else W.KERNEL_VALU)
    ctx.load(buf, w)
    seen = {}
    counts = []
    for _ in range(args.runs):
        n = ctx.run(thr)
        counts.append(n)
        st = ctx.rows()
        for a, b, s in st:
            seen.setdefault((a, b), []).append((s.d, s.d_prime, s.r2))
    print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("WLD_")}, "counts": counts,
                      "distinct_rows": len(seen)}))
    for (a, b), vals in list(seen.items())[:20]:
        ref = O.single_pair(buf[a], buf[b], w)
        t = O.all_pairs_dense_f64(np.stack([buf[a], buf[b]]), w)
        print(json.dumps({"a": a, "b": b, "times": len(vals), "gpu": vals[0], "oracle": ref,
                          "f64": [float(t[0][0, 1]), float(t[1][0, 1]), float(t[2][0, 1])]}))


if __name__ == "__main__":
    main()
