#!/usr/bin/env python3
"""Race screen for the MFMA kernel's LDS ring: both MFMA code paths compute
exact integer sums and the same f32 epilogue, so the ring path (fragment-major
codes through LDS) must reproduce the site-major path bit for bit.  Runs the
ring path repeatedly at a low threshold (tens of millions of rows) and counts
rows that differ from one site-major reference run."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402
import weightedld_amd._lib as _L  # noqa: E402
if os.environ.get("WLD_TOOL_LIB"):
    _L.LIB_PATH = os.path.abspath(os.environ["WLD_TOOL_LIB"])
import weightedld_amd as W  # noqa: E402
from weightedld_amd import dist as wdist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--thr", type=float, default=0.001)
    ap.add_argument("--runs", type=int, default=10)
    args = ap.parse_args()
    os.environ["WLD_NO_PREFILTER"] = "1"
    N, L, _, _ = bench.CONFIGS[args.config]
    buf = bench.synth(L, N)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    dev = torch.device("cuda", 0)
    os.environ["WLD_MFMA_LAYOUT"] = "rows"
    ref_ctx = W.Context(0, W.KERNEL_MFMA)
    ref_ctx.load(buf, w)
    os.environ.pop("WLD_MFMA_LAYOUT")
    n_ref = ref_ctx.run(args.thr)
    ref = wdist.pack_rows_device(ref_ctx, n_ref, dev)
    ring = W.Context(0, W.KERNEL_MFMA)
    ring.load(buf, w)
    out = []
    for _ in range(args.runs):
        n = ring.run(args.thr)
        got = wdist.pack_rows_device(ring, n, dev)
        where = []
        if n == n_ref:
            badm = (got != ref).any(dim=0)
            bad = int(badm.sum().item())
            if bad:
                idx = torch.nonzero(badm).flatten()[:4000].cpu().numpy()
                ab = ref[:2, idx].cpu().numpy().view("uint32")
                tiles = {}
                for a, b in zip(ab[0], ab[1]):
                    key = "%d,%d,w%d%d" % (a // 64, b // 64, (a % 64) // 32, (b % 64) // 32)
                    t = tiles.setdefault(key, {"n": 0, "rows": set(), "cols": set()})
                    t["n"] += 1
                    t["rows"].add(int(a % 32))
                    t["cols"].add(int(b % 32))
                where = [(k, v["n"], sorted(v["rows"]), len(v["cols"])) for k, v in
                         sorted(tiles.items(), key=lambda kv: -kv[1]["n"])[:6]]
                gd = got[2, idx[:4]].cpu().numpy().view("float32").tolist()
                rd = ref[2, idx[:4]].cpu().numpy().view("float32").tolist()
                where.append(("d_gpu_vs_ref", gd, rd))
        else:
            # row sets differ: locate the extra/missing (a, b) keys
            kg = got[0].long() * L + got[1].long()
            kr = ref[0].long() * L + ref[1].long()
            extra = kg[~torch.isin(kg, kr)]
            missing = kr[~torch.isin(kr, kg)]
            bad = int(extra.numel() + missing.numel())
            tiles = {}
            for k in torch.cat([extra, missing]).cpu().numpy()[:2000]:
                a, b = int(k) // L, int(k) % L
                key = "%d,%d,w%d%d,r%d" % (a // 64, b // 64, (a % 64) // 32, (b % 64) // 32, a % 32)
                tiles[key] = tiles.get(key, 0) + 1
            where = sorted(tiles.items(), key=lambda kv: -kv[1])[:8]
        out.append({"rows": n, "bad_rows": bad, "where": where})
    print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("WLD_")}, "ref_rows": n_ref,
                      "ring_runs": out}))


if __name__ == "__main__":
    main()
