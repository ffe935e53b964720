"""The N>1 step path with real device contexts at world 2-3 (one GPU).

Every rank is its own process owning real Contexts on device 0 and runs its
chunk-range shard (wld_shard_chunks) through ShardStep / PipelinedShardStep —
the bench's N>1 loop: wld_run_chunks_async on the library's stream, the
pipelined steps queued behind each other with wld_run_after, wld_run_wait,
the rows copied out with wld_rows_copy_device.  RCCL refuses two ranks on one
device, so the counts and rows travel as host tensors over gloo
(host_collectives=True); the device side is exactly the bench's.  Rank 0
checks every step's gathered rows against the unsharded oracle, bit for bit
(the default summation order is lib.rs's), over a threshold sequence in
which every rank, no rank or only some ranks have rows (lib.rs:635-679 split
over ranks and reassembled in reference order).
"""
import os
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import REPO
from test_dist import _free_port, ld_region_data

pytestmark = pytest.mark.gpu


def _gpu_step_worker(rank, world, port, L, N, thrs, mode, q, counts="collective"):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import torch
    import torch.distributed as dist

    import _oracle as O
    import weightedld_amd as W
    from weightedld_amd import dist as wdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        buf, w = ld_region_data(L, N, 5)
        lo, hi = wdist.shard_chunks(L, world, rank)
        depth = int(mode[0]) if mode != "step" else 1
        ctxs = [W.Context(0) for _ in range(depth)]
        for c in ctxs:
            c.load(buf, w)
        results = []
        xchg = wdist.HostCountExchange(rank, world) if counts == "shm" else None
        if mode == "step":
            step = wdist.ShardStep(ctxs[0], rank, world, dev, host_collectives=True, counts=xchg)
            results = [step(t, lo, hi) for t in thrs]
        else:
            pipe = wdist.PipelinedShardStep(ctxs, rank, world, dev, host_collectives=True,
                                            serialize_kernels="pair" if mode.endswith("pair") else False,
                                            counts=xchg)
            for t in thrs:
                r = pipe.submit(t, lo, hi)
                if r is not None:
                    results.append(r)
            results += pipe.drain_all()
        torch.cuda.synchronize()
        mine = [int(n) for n, _ in results]
        counts = [None] * world
        dist.all_gather_object(counts, mine)
        if rank == 0:
            ok = []
            for i, t in enumerate(thrs):
                ref = O.all_pairs(buf, w, np.float32(t), n_threads=4)
                got = wdist.unpack_rows(results[i][1])
                ok.append(len(got["site_a"]) == len(ref["site_a"]) and
                          all(np.array_equal(got[f], ref[f].astype(got[f].dtype)) if f in ("site_a", "site_b") else
                              np.array_equal(got[f].view(np.uint32), ref[f].view(np.uint32))
                              for f in wdist.ROW_FIELDS))
            q.put((ok, counts))
        else:
            assert all(r[1] is None for r in results)
        for c in ctxs:
            c.close()
        if xchg is not None:
            xchg.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("counts", ["collective", "shm"])
@pytest.mark.parametrize("mode", ["step", "2pair", "3pair", "2"])
@pytest.mark.parametrize("world", [2, 3])
def test_gpu_shard_steps_multi_rank(world, mode, counts):
    L, N = 1200, 200
    thrs = [0.0, 2.0, 0.5, 2.0, 0.0, 0.5, 0.5]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_step_worker, args=(r, world, port, L, N, thrs, mode, q, counts))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert all(c == 0 for c in codes), codes
    ok, counts = q.get(timeout=10)
    assert all(ok), ok
    per_step = list(zip(*counts))
    assert all(sum(c) == 0 for c, t in zip(per_step, thrs) if t == 2.0)
    assert any(0 < sum(1 for x in c if x) < world for c, t in zip(per_step, thrs) if t == 0.5)


def _shared_ctx_worker(port, q):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import torch
    import torch.distributed as dist

    import _oracle as O
    import weightedld_amd as W
    from weightedld_amd import dist as wdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        L, N = 1200, 200
        buf, w = ld_region_data(L, N, 5)
        ctxs = [W.Context(0) for _ in range(3)]
        for c in ctxs:
            c.load(buf, w)
        lo, hi = wdist.shard_chunks(L, 1, 0)
        pipe = wdist.PipelinedShardStep(ctxs, 0, 1, dev)
        single = wdist.ShardStep(ctxs[0], 0, 1, dev)
        same = single.stream is pipe.steps[0].stream
        ok = []
        refs = {t: O.all_pairs(buf, w, np.float32(t), n_threads=4) for t in (0.0, 0.5, 2.0)}

        def equal(res, t):
            got = wdist.unpack_rows(res[1])
            ref = refs[t]
            return len(got["site_a"]) == len(ref["site_a"]) and all(
                np.array_equal(got[f], ref[f].astype(got[f].dtype)) if f in ("site_a", "site_b") else
                np.array_equal(got[f].view(np.uint32), ref[f].view(np.uint32)) for f in wdist.ROW_FIELDS)

        for rnd in range(3):
            done = []
            for t in (0.5, 2.0, 0.0, 0.5):
                r = pipe.submit(t, lo, hi)
                if r is not None:
                    done.append(r)
            done += pipe.drain_all()
            ok += [equal(r, t) for r, t in zip(done, (0.5, 2.0, 0.0, 0.5))]
            for t in (0.0, 0.5, 2.0):  # the single step on the pipeline's first context, between pipelined runs
                ok.append(equal(single(t, lo, hi), t))
        torch.cuda.synchronize()
        pipe.close()
        single.close()
        for c in reversed(ctxs):
            c.close()
        q.put((same, ok))
    finally:
        dist.destroy_process_group()


def test_shard_step_beside_pipeline_on_one_context():
    """a ShardStep made on a context a PipelinedShardStep also
    steps (the bench's stats and checked steps at N>1) shares that context's
    stream, so its count all_gather and pinned copy are ordered behind its
    own scan; interleaved single and pipelined steps, over RCCL in a group of
    one, give the oracle's rows every time (thresholds with all, some and no
    rows)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_shared_ctx_worker, args=(_free_port(), q))
    p.start()
    p.join(timeout=240)
    if p.is_alive():
        p.kill()
    assert p.exitcode == 0, p.exitcode
    same, ok = q.get(timeout=10)
    assert same and all(ok) and len(ok) == 21, (same, ok)
