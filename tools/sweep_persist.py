#!/usr/bin/env python3
"""Row-count determinism sweep of the persistent MFMA kernel at thr 0.05 on
synthetic data whose reference has (almost) no rows: extra rows = corruption."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402,F401

import weightedld_amd._lib as _L  # noqa: E402
if os.environ.get("WLD_TOOL_LIB"):
    _L.LIB_PATH = os.path.abspath(os.environ["WLD_TOOL_LIB"])
import weightedld_amd as W  # noqa: E402
from test_gpu_parity import synth  # noqa: E402

os.environ["WLD_NO_PREFILTER"] = "1"
for L in [int(x) for x in sys.argv[1].split(",")]:
    buf = synth(L, 2000, 77)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    os.environ["WLD_MFMA_LAYOUT"] = "rows"
    ref = W.Context(0, W.KERNEL_MFMA)
    ref.load(buf, w)
    os.environ.pop("WLD_MFMA_LAYOUT")
    n_ref = ref.run(0.05)
    del ref
    ctx = W.Context(0, W.KERNEL_MFMA)
    ctx.load(buf, w)
    for cfg in sys.argv[2].split(";"):
        for kv in cfg.split(","):
            if "=" in kv:
                k, v = kv.split("=")
                os.environ[k] = v
        ns = [ctx.run(0.05) for _ in range(3)]
        print(json.dumps({"lib": os.environ.get("WLD_TOOL_LIB"), "L": L, "cfg": cfg, "n_ref": n_ref, "n": ns}),
              flush=True)
        for kv in cfg.split(","):
            if "=" in kv:
                os.environ.pop(kv.split("=")[0], None)
