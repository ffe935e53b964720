#!/usr/bin/env python3
"""Debug probe: rows of the candidate-pair path (WLD_OPT_SCREEN 4) that differ
from the oracle on one input, for the given library builds (one child process
each); prints the one-sided rows with GPU and oracle values.
    python tools/probes/ref_pairs_debug.py [lib.so ...]"""
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(lib):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import weightedld_amd._lib as WL
    if lib != "default":
        WL.LIB_PATH = os.path.abspath(lib)
    import _oracle as O
    import weightedld_amd as W
    from test_gpu_screen import ld_blocks
    buf = ld_blocks(900, 257, 3)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    d, dp, r2, valid = O.all_pairs_dense(buf, w)
    ref = O.all_pairs(buf, w, np.float32(0.002))
    kr = set(zip(ref["site_a"].tolist(), ref["site_b"].tolist()))
    for rep in range(3):
        ctx = W.Context(0, W.KERNEL_AUTO)
        ctx.set_option("screen", 4)
        ctx.load(buf, w)
        n = ctx.run(0.002)
        st = ctx.stats()
        rows = ctx.rows()
        kg = set(zip(rows.site_a.tolist(), rows.site_b.tolist()))
        print(lib, "rep", rep, "rows", n, len(ref["site_a"]), "cand", st["candidate_pairs"], "only gpu",
              len(kg - kr), "only ref", len(kr - kg), flush=True)
        ga = {k: i for i, k in enumerate(zip(rows.site_a.tolist(), rows.site_b.tolist()))}
        for k in sorted(kg - kr)[:6]:
            i = ga[k]
            print("  gpu-only", k, "gpu r2", rows.r2[i], "oracle r2", r2[k], "valid", valid[k], flush=True)
        for k in sorted(kr - kg)[:6]:
            print("  ref-only", k, "oracle r2", r2[k], flush=True)
        common = sorted(kg & kr)
        ib = {k: i for i, k in enumerate(zip(ref["site_a"].tolist(), ref["site_b"].tolist()))}
        bad = sum(1 for k in common if rows.r2[ga[k]].view(np.uint32) != ref["r2"][ib[k]].view(np.uint32))
        print("  common rows with different r2 bits:", bad, flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
    else:
        for lib in (sys.argv[1:] or ["default"]):
            subprocess.run([sys.executable, __file__, "--child", lib], timeout=250)
