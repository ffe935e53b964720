"""Per-step host overhead of the N>1 bench step, simulated on one GPU: the
kernel over one rank's 1/8 shard of C4, then the count exchange of
weightedld_amd.dist.RowGather through a world-1 RCCL group (the collective
path forced), against the old list-based all_gather and the bare run.
    python tools/step_sim.py"""
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import weightedld_amd as W  # noqa: E402
from weightedld_amd import dist as wdist  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
N, L, thr, _ = bench.CONFIGS["c4"]
buf = bench.synth(L, N)
w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
ctx = W.Context(0)
ctx.load(buf, w)
b, e = ctx.shard_chunks(L, 8, 0)
rg = wdist.RowGather(0, 1, dev)
rg.world = 2  # force the collective path (the count buffers stay world-1 sized)
ss = wdist.ShardStep(ctx, 0, 1, dev)  # world-1 group: the same collective calls


def old_gather(packed):
    cnt = torch.tensor([packed.shape[1]], dtype=torch.int64, device=dev)
    cnts = [torch.zeros_like(cnt)]
    dist.all_gather(cnts, cnt)
    return [int(c) for c in torch.cat(cnts).cpu().tolist()]


variants = {
    "run only": lambda: ctx.run_chunks(thr, b, e),
    "run + RowGather": lambda: rg(wdist.pack_rows_device(ctx, ctx.run_chunks(thr, b, e), dev)),
    "run + old all_gather": lambda: old_gather(wdist.pack_rows_device(ctx, ctx.run_chunks(thr, b, e), dev)),
    "ShardStep (async)": lambda: ss(thr, b, e),
}
for name, f in variants.items():
    for _ in range(20):
        f()
for rnd in range(2):
    for name, f in variants.items():
        wall, kern = [], []
        for _ in range(50):
            t0 = time.perf_counter()
            f()
            wall.append((time.perf_counter() - t0) * 1e3)
            kern.append(ctx.stats()["pair_kernel_ms"])
        print("%-22s wall %.3f ms  kernel %.3f ms  overhead %.3f ms" %
              (name, np.median(wall), np.median(kern), np.median(wall) - np.median(kern)), flush=True)
dist.destroy_process_group()
