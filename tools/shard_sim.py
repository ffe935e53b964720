"""Predicts the strong-scaling efficiency of the N-GPU bench from one GPU:
runs every rank's shard (row-block or chunk-range split) of a config one
after another on cuda:0 and reports each shard's pair-kernel time (HIP
events), the slowest shard against full/N, and the implied efficiency of the
kernel phase.  The real N-GPU run adds the count all_gather per step.
    python tools/shard_sim.py [--config c4] [--worlds 2,4,8] [--reps 5]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import weightedld_amd as W  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    N, L, thr, _ = bench.CONFIGS[args.config]
    buf = bench.synth(L, N)
    ss = W.SiteSet.from_buffer(buf)
    kept = ss.filter_sites_of_interest()
    w = W.henikoff_weights(kept)
    ctx = W.Context(0)
    ctx.load(buf, w)

    def timed(run):
        for _ in range(2):
            run()
        ms = []
        for _ in range(args.reps):
            run()
            ms.append(ctx.stats()["pair_kernel_ms"])
        return float(np.median(ms))

    full = timed(lambda: ctx.run(thr))
    out = {"config": args.config, "full_kernel_ms": full, "worlds": {}}
    for world in [int(x) for x in args.worlds.split(",")]:
        for split in ("rows", "chunks"):
            shard_ms, shard_pairs = [], []
            for r in range(world):
                if split == "rows":
                    b, e = ctx.shard_chunk_rows(L, world, r)
                    shard_ms.append(timed(lambda: ctx.run(thr, b, e)))
                else:
                    b, e = ctx.shard_chunks(L, world, r)
                    shard_ms.append(timed(lambda: ctx.run_chunks(thr, b, e)))
                shard_pairs.append(ctx.stats()["pairs"])
            eff = full / world / max(shard_ms)
            out["worlds"]["%d/%s" % (world, split)] = {
                "shard_kernel_ms": [round(x, 4) for x in shard_ms], "max_ms": max(shard_ms),
                "pairs_max_over_mean": max(shard_pairs) / (sum(shard_pairs) / world), "kernel_efficiency": eff}
            print("world %d %-6s max shard %.3f ms (ideal %.3f) eff %.3f pairs max/mean %.4f" %
                  (world, split, max(shard_ms), full / world, eff, max(shard_pairs) / (sum(shard_pairs) / world)),
                  flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
