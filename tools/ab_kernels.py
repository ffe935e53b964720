#!/usr/bin/env python3
"""Interleaved A/B timing of pair-kernel variants in one process (GPU).

Variants are selected through the library's experiment knobs:
  WLD_MFMA_LAYOUT=rows   site-major code reads instead of the fragment-major copy
  WLD_NO_PREFILTER=1     no exact-integer r2 prefilter before the f32 epilogue
Prints one JSON line per variant with median/min pair-kernel ms (HIP events).
"""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402,F401  (one HIP runtime: torch's)

import bench  # noqa: E402
import weightedld_amd as W  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variants", default="rows,rows+pf,frag,frag+pf,valu")
    args = ap.parse_args()
    N, L, thr, _ = bench.CONFIGS[args.config]
    buf = bench.synth(L, N)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    ctxs = {}
    for v in args.variants.split(","):
        os.environ.pop("WLD_MFMA_LAYOUT", None)
        if v.startswith("rows"):
            os.environ["WLD_MFMA_LAYOUT"] = "rows"
        ctx = W.Context(0, W.KERNEL_VALU if v == "valu" else W.KERNEL_MFMA)
        ctx.load(buf, w)
        ctxs[v] = ctx
    os.environ.pop("WLD_MFMA_LAYOUT", None)
    times = {v: [] for v in ctxs}
    rows = {}
    for _ in range(args.rounds):
        for v, ctx in ctxs.items():
            if v.endswith("+pf") or v == "valu":
                os.environ.pop("WLD_NO_PREFILTER", None)
            else:
                os.environ["WLD_NO_PREFILTER"] = "1"
            for _ in range(args.reps):
                rows[v] = ctx.run(thr)
                times[v].append(ctx.stats()["pair_kernel_ms"])
    os.environ.pop("WLD_NO_PREFILTER", None)
    for v, t in times.items():
        pairs = L * (L - 1) // 2
        print(json.dumps({"config": args.config, "variant": v, "median_ms": statistics.median(t), "min_ms": min(t),
                          "pairs_per_s": pairs / (statistics.median(t) * 1e-3), "rows": rows[v], "n": len(t)}))


if __name__ == "__main__":
    main()
