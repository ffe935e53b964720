"""Multi-rank (gloo, CPU) tests of the N>1 path: shard planning, per-shard
rows in reference order, gather to rank 0 and reassembly.

Each rank computes its shard's rows with the CPU oracle (standing in for the
rows its GPU leaves in HBM; the GPU side of a shard is covered by
test_gpu_parity.py::test_sharded_runs_concatenate_to_reference_order) and the
product gather (weightedld_amd.dist) reassembles them; rank 0 checks the
result equals the unsharded reference-order rows exactly.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, L, N, thr, q, by_chunk=False):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import torch.distributed as dist

    import _oracle as O
    from weightedld_amd import dist as wdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(42)
        buf = rng.integers(0, 5, size=(L, N)).astype(np.uint8)
        w = rng.random(N).astype(np.float32)
        if by_chunk:  # the bench's split: contiguous chunk ranges (wld_shard_chunks)
            lo, hi = wdist.shard_chunks(L, world, rank)
        else:  # whole chunk rows (wld_shard_chunk_rows)
            rb, re_ = wdist.shard_rows(L, world, rank)
            n = (L + 255) // 256
            lin = lambda r, c: (n - 1 - r) * (n - r) // 2 + (c - r)  # noqa: E731
            lo, hi = (lin(re_ - 1, re_ - 1), lin(rb, rb) + (n - rb)) if re_ > rb else (0, 0)
        mine = O.all_pairs(buf, w, thr, n_threads=2, chunk_lo=lo, chunk_hi=hi) if hi > lo else \
            {f: np.zeros(0, dtype=np.float32 if f in ("d", "d_prime", "r2") else np.uint64) for f in wdist.ROW_FIELDS}
        out = wdist.gather_rows(wdist.pack_rows_host(mine), rank, world)
        if rank == 0:
            got = wdist.unpack_rows(out)
            ref = O.all_pairs(buf, w, thr, n_threads=2)
            ok = all(np.array_equal(got[f], ref[f].astype(got[f].dtype)) for f in wdist.ROW_FIELDS)
            q.put((ok, len(got["site_a"]), len(ref["site_a"])))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("by_chunk", [False, True], ids=["rows", "chunks"])
@pytest.mark.parametrize("world,L,N,thr", [(2, 1300, 24, 0.0), (3, 900, 16, 0.02), (2, 300, 12, 2.0), (4, 600, 8, 0.0)])
def test_gloo_shard_gather_matches_unsharded(world, L, N, thr, by_chunk):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, L, N, thr, q, by_chunk)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ok, n_got, n_ref = q.get(timeout=10)
    assert ok and n_got == n_ref
