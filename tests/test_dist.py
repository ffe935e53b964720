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


class OracleShardContext:
    """Stand-in for a device Context in the N>1 step path (ShardStep,
    PipelinedShardStep): run_chunks_async computes the chunk range's rows with
    the oracle and writes the row count (int64) to the given address, as
    wld_run_chunks_async does on the device; rows_copy_device copies them to
    the given (host) addresses, as wld_rows_copy_device does."""

    def __init__(self, buf, w):
        self.buf, self.w, self.rows, self.pending = buf, w, None, False

    def stream_ptr(self):
        return 0

    def run_chunks_async(self, thr, lo, hi, d_count_ptr=None):
        import ctypes

        import _oracle as O
        assert not self.pending, "run_chunks_async twice without run_wait"
        self.rows = O.all_pairs(self.buf, self.w, thr, n_threads=2, chunk_lo=lo, chunk_hi=hi)
        self.pending = True
        if d_count_ptr:
            ctypes.c_int64.from_address(d_count_ptr).value = len(self.rows["r2"])

    def run_after(self, prev):  # device-side ordering: program order on the host
        pass

    def run_wait(self):
        assert self.pending, "run_wait with nothing in flight"
        self.pending = False
        return len(self.rows["r2"])

    def rows_copy_device(self, a, b, d, dp, r2):
        import ctypes
        for ptr, f, dt in ((a, "site_a", np.uint32), (b, "site_b", np.uint32), (d, "d", np.float32),
                           (dp, "d_prime", np.float32), (r2, "r2", np.float32)):
            col = np.ascontiguousarray(self.rows[f].astype(dt))
            if ptr and col.size:
                ctypes.memmove(ptr, col.ctypes.data, col.nbytes)


def ld_region_data(L, N, seed):
    """Random sites (no pair near r2 0.5 at this N) plus one block of 40
    linked sites near the end of the site order: at r2_threshold 0.5 only the
    shards holding those sites' chunks have rows."""
    rng = np.random.default_rng(seed)
    buf = rng.integers(0, 2, size=(L, N)).astype(np.uint8)  # 2 symbols: every site has maj+min
    f = rng.random(N) < 0.4
    for s in range(L - 60, L - 20):
        buf[s] = np.where(f ^ (rng.random(N) < 0.03), 1, 0)
    return buf, rng.random(N).astype(np.float32) + 0.2


def _step_worker(rank, world, port, L, N, thrs, pipelined, q, counts="collective"):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import torch.distributed as dist

    import _oracle as O
    from weightedld_amd import dist as wdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        buf, w = ld_region_data(L, N, 5)
        lo, hi = wdist.shard_chunks(L, world, rank)
        results = []
        xchg = wdist.HostCountExchange(rank, world) if counts == "shm" else None
        if pipelined:
            depth, mode = int(str(pipelined)[0]), ("pair" if str(pipelined).endswith("pair") else False)
            pipe = wdist.PipelinedShardStep([OracleShardContext(buf, w) for _ in range(depth)], rank, world,
                                            "cpu", serialize_kernels=mode, counts=xchg)
            for t in thrs:
                r = pipe.submit(t, lo, hi)
                if r is not None:
                    results.append(r)
            results += pipe.drain_all()
            assert pipe.drain() is None
        else:
            step = wdist.ShardStep(OracleShardContext(buf, w), rank, world, "cpu", counts=xchg)
            results = [step(t, lo, hi) for t in thrs]
        mine = [int(n) for n, _ in results]
        counts = [None] * world
        dist.all_gather_object(counts, mine)
        if xchg is not None:
            xchg.close()
        if rank == 0:
            ok = []
            for i, t in enumerate(thrs):
                ref = O.all_pairs(buf, w, t, n_threads=2)
                got = wdist.unpack_rows(results[i][1])
                ok.append(all(np.array_equal(got[f], ref[f].astype(got[f].dtype)) for f in wdist.ROW_FIELDS))
            q.put((ok, counts))
        else:
            assert all(r[1] is None for r in results)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("counts", ["collective", "shm"])
@pytest.mark.parametrize("pipelined", [0, 2, 3, "3pair"], ids=["step", "pipelined2", "pipelined3", "pipelined3pair"])
@pytest.mark.parametrize("world", [2, 3, 4])
def test_gloo_shard_steps_match_unsharded(world, pipelined, counts):
    """ShardStep / PipelinedShardStep (the bench's N>1 step path) at world
    2-4 under gloo: per step, the count exchange, the row gather issued only
    when some rank has rows, and (pipelined) step i-1's gather issued after
    step i's count exchange; depth 3: two steps in flight) — every step's gathered rows equal the unsharded
    oracle's, in reference order, with threshold sequences where no rank,
    one rank or every rank has rows, and nothing deadlocks; the row counts
    exchanged by a collective or through host shared memory
    (HostCountExchange)."""
    L, N = 1200, 200
    thrs = [0.0, 2.0, 0.5, 2.0, 0.0, 0.5, 0.5]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_step_worker, args=(r, world, port, L, N, thrs, pipelined, q, counts))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ok, counts = q.get(timeout=10)
    assert all(ok), ok
    # the planted block gives rows at 0.5 to some ranks only; 2.0 to none
    per_step = list(zip(*counts))
    assert all(sum(c) == 0 for c, t in zip(per_step, thrs) if t == 2.0)
    assert any(0 < sum(1 for x in c if x) < world for c, t in zip(per_step, thrs) if t == 0.5)


# ---- world 8 at BASELINE configs 4 and 5's chunk counts ----

def test_world8_shards_balanced_at_c4_c5():
    """wld_shard_chunks at N=8 over C4 (20,000 sites: 3,160 chunks) and C5
    (50,000: 19,306 chunks): contiguous, covering, in descending-rank
    position (shard k the k-th range from the end), pair counts within 1% of
    the mean (lib.rs:615-634's chunk sequence, split at chunk granularity)."""
    sys.path.insert(0, REPO)
    from weightedld_amd import dist as wdist
    from weightedld_amd.api import Context
    for L, nchunks in ((20000, 3160), (50000, 19306)):
        assert Context.chunks(L) == nchunks
        rng = [wdist.shard_chunks(L, 8, r) for r in range(8)]
        assert rng[7][0] == 0 and rng[0][1] == nchunks
        for r in range(7):
            assert rng[r + 1][1] == rng[r][0]  # rank r + 1's range ends where rank r's begins
        pairs = [Context.pairs_in_chunks(L, b, e) for b, e in rng]
        assert sum(pairs) == L * (L - 1) // 2
        assert max(pairs) / (sum(pairs) / 8) <= 1.01, pairs


class CachedOracleContext(OracleShardContext):
    """OracleShardContext computing each chunk range's rows once, at the
    lowest threshold of the run (shared by the pipeline's contexts), and
    each step's rows as the strict r2 > thr subset of them (lib.rs:660) —
    the same rows the oracle gives at thr."""

    def __init__(self, buf, w, base_thr, cache):
        super().__init__(buf, w)
        self.base, self.cache = np.float32(base_thr), cache

    def run_chunks_async(self, thr, lo, hi, d_count_ptr=None):
        import ctypes

        import _oracle as O
        assert not self.pending and np.float32(thr) >= self.base
        if (lo, hi) not in self.cache:
            self.cache[(lo, hi)] = O.all_pairs(self.buf, self.w, self.base, n_threads=1, chunk_lo=lo, chunk_hi=hi)
        full = self.cache[(lo, hi)]
        m = full["r2"] > np.float32(thr)
        self.rows = {f: full[f][m] for f in ROW_KEYS}
        self.pending = True
        if d_count_ptr:
            ctypes.c_int64.from_address(d_count_ptr).value = len(self.rows["r2"])


ROW_KEYS = ("site_a", "site_b", "d", "d_prime", "r2")


def c4_world8_data():
    """C4's site count with N = 32 binary sequences (random pairs reach r2
    0.5 about once in 16,000: rows on every rank) and one block of exact
    copies near the middle of the site order (r2 = 1: at 0.999 only the
    shard holding the block's chunks has rows)."""
    rng = np.random.default_rng(808)
    L, N = 20000, 32
    buf = rng.integers(0, 2, size=(L, N)).astype(np.uint8)
    for s in range(9001, 9006):
        buf[s] = buf[9000]
    return buf, np.full(N, 1.0, dtype=np.float32) + rng.random(N).astype(np.float32)


class PlantedRowsContext(OracleShardContext):
    """A shard context whose rows are a closed-form set of passing pairs (at
    C5's 50,000 sites an oracle pass does not fit a CPU test): 3,000 pairs
    (a < b) with r2 drawn uniformly, some in every rank's range; a chunk
    range's rows are the pairs in its chunks with r2 > thr, in the reference
    order (chunk linear index ascending: chunk rows descend; inside a chunk a,
    then b, lib.rs:623-683).  The reference is the whole set in that order."""

    L = 50000

    @staticmethod
    def table():
        rng = np.random.default_rng(5050)
        L = PlantedRowsContext.L
        a = rng.integers(0, L - 1, size=3000)
        b = np.minimum(L - 1, a + 1 + rng.integers(0, 4000, size=3000))
        a, b = np.unique(np.stack([a, b], 1), axis=0).T
        n = (L + 255) // 256
        row, col = a // 256, b // 256
        lin = (n - 1 - row) * (n - row) // 2 + (col - row)
        order = np.lexsort((b, a, lin))
        r2 = rng.random(len(a)).astype(np.float32)
        return {"lin": lin[order], "site_a": a[order].astype(np.uint64), "site_b": b[order].astype(np.uint64),
                "d": (r2 * 0.25)[order], "d_prime": np.sqrt(r2)[order].astype(np.float32), "r2": r2[order]}

    def __init__(self):
        super().__init__(None, None)
        self.t = self.table()

    def run_chunks_async(self, thr, lo, hi, d_count_ptr=None):
        import ctypes
        assert not self.pending
        m = (self.t["lin"] >= lo) & (self.t["lin"] < hi) & (self.t["r2"] > np.float32(thr))
        self.rows = {f: self.t[f][m] for f in ROW_KEYS}
        self.pending = True
        if d_count_ptr:
            ctypes.c_int64.from_address(d_count_ptr).value = len(self.rows["r2"])


def _world8_worker(rank, world, port, kind, pipelined, thrs, q, counts="collective"):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import torch.distributed as dist

    import _oracle as O
    from weightedld_amd import dist as wdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if kind == "c4":
            buf, w = c4_world8_data()
            L = buf.shape[0]
            cache = {}
            make = lambda: CachedOracleContext(buf, w, min(thrs), cache)  # noqa: E731
        else:
            L = PlantedRowsContext.L
            make = PlantedRowsContext
        lo, hi = wdist.shard_chunks(L, world, rank)
        xchg = wdist.HostCountExchange(rank, world) if counts == "shm" else None
        if pipelined:
            pipe = wdist.PipelinedShardStep([make() for _ in range(pipelined)], rank, world, "cpu", counts=xchg)
            results = []
            for t in thrs:
                r = pipe.submit(t, lo, hi)
                if r is not None:
                    results.append(r)
            results += pipe.drain_all()
        else:
            step = wdist.ShardStep(make(), rank, world, "cpu", counts=xchg)
            results = [step(t, lo, hi) for t in thrs]
        mine = [int(n) for n, _ in results]
        counts = [None] * world
        dist.all_gather_object(counts, mine)
        if xchg is not None:
            xchg.close()
        if rank == 0:
            if kind == "c4":
                base = O.all_pairs(buf, w, np.float32(min(thrs)), n_threads=8)
            else:
                base = PlantedRowsContext.table()
            ok = []
            for i, t in enumerate(thrs):
                m = base["r2"] > np.float32(t)
                got = wdist.unpack_rows(results[i][1])
                ok.append(all(np.array_equal(got[f], base[f][m].astype(got[f].dtype)) for f in ROW_KEYS))
            q.put((ok, counts))
        else:
            assert all(r[1] is None for r in results)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("counts", ["collective", "shm"])
@pytest.mark.parametrize("kind", ["c4", "c5"])
@pytest.mark.parametrize("pipelined", [0, 3], ids=["step", "pipelined3"])
def test_gloo_world8_steps(kind, pipelined, counts):
    """The driver's N=8 path before its SCALE run: eight gloo ranks, each
    with its chunk range of BASELINE config 4 (3,160 chunks; oracle-backed
    contexts, N = 32) or config 5 (19,306 chunks; closed-form rows), through
    ShardStep and the three-context PipelinedShardStep.  Thresholds where
    every rank, no rank and only some ranks have rows; every step's gathered
    rows equal the unsharded reference's, in reference order, bit for bit
    (lib.rs:634-679's collect, eight-way)."""
    thrs = [0.5, 2.0, 0.999, 0.5, 2.0, 0.999] if kind == "c4" else [0.0, 2.0, 0.9995, 0.3, 2.0, 0.9995]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_world8_worker, args=(r, 8, port, kind, pipelined, thrs, q, counts))
             for r in range(8)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ok, counts = q.get(timeout=10)
    assert all(ok), ok
    per_step = list(zip(*counts))
    for c, t in zip(per_step, thrs):
        nz = sum(1 for x in c if x)
        if t == 2.0:
            assert nz == 0, (t, c)
        elif t in (0.5, 0.0, 0.3):
            assert nz == 8, (t, c)
        else:
            assert 0 < nz < 8, (t, c)
