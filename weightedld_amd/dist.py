"""Multi-GPU sharding of the pair space and the gather of passing rows.

The L^2 pair space is split into contiguous runs of the reference's 256x256
chunk sequence (lib.rs:615-634, triu_index order), balanced by pair count at
single-chunk granularity, one run per rank (one process per GPU); the coarser
chunk-row split (shard_rows) is kept for callers that want whole rows.  Pairs are independent, so ranks exchange nothing while computing.
Each rank leaves its rows on its GPU in reference order; the only collective is
the final gather of those rows to rank 0 (RCCL over xGMI with the "nccl"
backend; gloo in the CPU tests).  Because chunk rows DESCEND in the reference's
triu_index order (lib.rs:623-632), rank 0 concatenates the shards in
descending rank order.
"""
import collections
import contextlib

import numpy as np

from .api import Context

ROW_FIELDS = ("site_a", "site_b", "d", "d_prime", "r2")


def shard_rows(n_sites, world, rank):
    """Chunk rows [begin, end) of this rank (balanced pair counts)."""
    return Context.shard_chunk_rows(n_sites, world, rank)


def shard_chunks(n_sites, world, rank):
    """Linear chunk range [begin, end) of this rank (balanced pair counts)."""
    return Context.shard_chunks(n_sites, world, rank)


def pack_rows_device(ctx, n, device):
    """The last run's rows as one [5, n] int32 tensor on `device` (floats bit-cast).
    Every element is overwritten by the copy (synchronous on the context's
    stream), so the buffer needs no initialising kernel on torch's stream."""
    import torch

    packed = torch.empty((5, max(n, 0)), dtype=torch.int32, device=device)
    if n:
        ctx.rows_copy_device(*(packed[i].data_ptr() for i in range(5)))
    return packed


def pack_rows_host(store):
    """A PairStore (host numpy) as a [5, n] int32 tensor (floats bit-cast)."""
    import torch

    cols = [np.ascontiguousarray(getattr(store, f)) for f in ROW_FIELDS] if not isinstance(store, dict) else \
        [np.ascontiguousarray(store[f]) for f in ROW_FIELDS]
    arr = np.stack([c.astype(np.uint32).view(np.int32) if c.dtype.kind == "u" else c.view(np.int32)
                    for c in cols]) if len(cols[0]) else np.zeros((5, 0), dtype=np.int32)
    return torch.from_numpy(np.ascontiguousarray(arr))


def unpack_rows(packed):
    """[5, n] int32 tensor -> dict of numpy columns."""
    a = packed.cpu().numpy()
    return {"site_a": a[0].view(np.uint32), "site_b": a[1].view(np.uint32), "d": a[2].view(np.float32),
            "d_prime": a[3].view(np.float32), "r2": a[4].view(np.float32)}


class RowGather:
    """Per-step gather of every rank's [5, n_r] rows to rank 0, with the
    count exchange on persistent buffers: one all_gather_into_tensor of the
    int64 counts (no host-to-device tensor build, no list of outputs) and one
    host read of the result; only when some rank has rows, one group of
    exact-size point-to-point transfers: each rank with rows
    sends its n_r rows, rank 0 receives each into a buffer of that size
    (batch_isend_irecv: one RCCL group; no padding to the largest count).
    Rank 0 gets the [5, sum n_r] concatenation in reference order (shards in
    descending rank order), other ranks None."""

    def __init__(self, rank, world, device, group=None):
        import torch

        self.rank, self.world, self.group, self.device = rank, world, group, device
        self.cnt = torch.zeros(1, dtype=torch.int64, device=device)
        self.cnts = torch.zeros(world, dtype=torch.int64, device=device)

    def __call__(self, packed, counts=None):
        """counts: the ranks' row counts when already exchanged (ShardStep)."""
        import torch
        import torch.distributed as dist

        if self.world == 1:
            return packed
        if counts is None:
            self.cnt.fill_(packed.shape[1])
            dist.all_gather_into_tensor(self.cnts, self.cnt, group=self.group)
            counts = self.cnts.tolist()  # the one host sync of a step without rows
        counts = [int(c) for c in counts]
        if max(counts) == 0:
            return packed[:, :0] if self.rank == 0 else None
        peer = (lambda r: dist.get_global_rank(self.group, r)) if self.group is not None else (lambda r: r)
        if self.rank != 0:
            n = counts[self.rank]
            if n:
                assert packed.shape[1] >= n, (packed.shape, n)
                for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, packed[:, :n].contiguous(), peer(0),
                                                            group=self.group)]):
                    w.wait()
            return None
        parts = {0: packed[:, :counts[0]]}
        ops = []
        for r in range(1, self.world):
            if counts[r]:
                parts[r] = torch.empty((5, counts[r]), dtype=torch.int32, device=packed.device)
                ops.append(dist.P2POp(dist.irecv, parts[r], peer(r), group=self.group))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        return torch.cat([parts[r] for r in reversed(range(self.world)) if r in parts], dim=1)


class HostCountExchange:
    """The per-step row-count exchange of ranks on one host through a block
    of host shared memory instead of a collective: each rank publishes its
    step's row count (known on the host once its own pass has completed,
    wld_run_wait) and reads every rank's.  One exchange costs a few
    microseconds of host time where the RCCL count all_gather, its stream
    scope, event and pinned copy cost ~30; the rows themselves
    still travel by the collective backend (RowGather).  Slots are
    double-buffered by step parity: a rank can publish step k + 2 only after
    every rank has published step k + 1, i.e. after every rank has read step
    k.  Within a slot the count is stored before the step number and read
    after it (x86-64: stores and loads are not reordered among themselves).
    Built collectively (rank 0 creates the block and broadcasts its name);
    all ranks must share the host."""

    def __init__(self, rank, world, group=None):
        import torch.distributed as dist
        from multiprocessing import resource_tracker, shared_memory

        self.rank, self.world, self.seq = rank, world, 0
        name = [None]
        if rank == 0:
            self.shm = shared_memory.SharedMemory(create=True, size=2 * 2 * 8 * world)
            np.ndarray((2, world, 2), dtype=np.int64, buffer=self.shm.buf)[:] = -1
            name[0] = self.shm.name
        if world > 1:
            dist.broadcast_object_list(name, src=0, group=group)
        if rank != 0:
            self.shm = shared_memory.SharedMemory(name=name[0])
            # (the creator owns the block: no second tracker unlinks it at exit)
            resource_tracker.unregister(self.shm._name, "shared_memory")
        self.slots = np.ndarray((2, world, 2), dtype=np.int64, buffer=self.shm.buf)  # [parity][rank][count, step]
        if world > 1:
            dist.barrier(group=group)  # every rank attached before the creator may unlink at close

    def __call__(self, count, timeout_s=300.0):
        self.seq += 1
        s = self.slots[self.seq & 1]
        s[self.rank, 0] = count
        s[self.rank, 1] = self.seq
        steps = s[:, 1]
        spins = 0
        while steps.min() < self.seq:
            spins += 1
            if spins & 0xFFFF == 0:  # (a rank that died never publishes: fail instead of spinning forever)
                import time
                if spins == 0x10000:
                    self._t0 = time.monotonic()
                elif time.monotonic() - self._t0 > timeout_s:
                    raise RuntimeError("HostCountExchange: step %d: ranks %s did not publish within %.0f s" % (
                        self.seq, np.nonzero(steps < self.seq)[0].tolist(), timeout_s))
        return s[:, 0].tolist()

    def close(self):
        if self.shm is not None:
            self.slots = None
            self.shm.close()
            if self.rank == 0:
                self.shm.unlink()
            self.shm = None


class _HostStream:
    """Stand-in for the context's stream when the step runs on the CPU (the
    gloo rehearsal of the N>1 path in tests/test_dist.py): ordering is program
    order, so waits are no-ops."""

    def wait_event(self, event):
        pass


class _HostEvent:
    def record(self, stream=None):
        pass


def _stream_scope(stream):
    import torch

    return contextlib.nullcontext() if isinstance(stream, _HostStream) else torch.cuda.stream(stream)


class ShardStep:
    """One all_weighted_ld_pairs pass over this rank's chunk range with the
    row gather to rank 0, in one host wait when no rank has rows: the pair
    kernel and the row count are enqueued on the context's stream
    (wld_run_chunks_async), the count all_gather is ordered after them on that
    same stream, and one device-to-host read of the gathered counts completes
    both.  Returns (rows on this rank, gathered [5, n] rows on rank 0 / None).

    ctx is anything with the Context methods the step uses
    (run_chunks_async, run_wait, rows_copy_device, set_stream); with a CPU
    `device` the step runs in program order on host tensors (gloo).
    host_collectives=True keeps the device's kernels and the context's
    stream but exchanges counts and rows as host tensors (gloo): several
    ranks on one GPU, where RCCL refuses a duplicate device (the multi-rank
    GPU test); the count then reaches the host before its all_gather."""

    def __init__(self, ctx, rank, world, device, group=None, host_collectives=False, counts=None):
        import torch

        self.ctx = ctx
        # counts: a HostCountExchange (ranks on one host): the row counts are
        # exchanged through host shared memory after the pass, no count collective
        self.xchg = counts
        device = torch.device(device)
        self.host = host_collectives and device.type == "cuda"
        self.gather = RowGather(rank, world, torch.device("cpu") if self.host else device, group)
        self.cnt_dev = torch.zeros(1, dtype=torch.int64, device=device) if self.host else None
        self.device = device
        # The context runs on a torch-owned stream (wld_set_stream): the count
        # collective, its event and the pinned copy below are recorded on a
        # stream that outlives every torch object referencing it (torch never
        # destroys its pool streams), whatever order the context and those
        # objects are released in.  (Round 4 recorded them on the context's own
        # stream, wrapped as an ExternalStream, and the process crashed at exit,
        # profiles/r04i/: the context was destroyed by its finalizer at
        # interpreter shutdown, in no set order against the torch event and
        # pinned-memory block recorded on the stream it destroyed.)
        # One stream per context: a second step object on the same context
        # (the bench's ShardStep beside its PipelinedShardStep) reuses the
        # stream the first bound, so every step on that context, its count
        # collective and its pinned copy stay ordered on one stream.
        if device.type == "cuda":
            self.stream = getattr(ctx, "_shard_step_stream", None)
            if self.stream is None:
                self.stream = torch.cuda.Stream(device=device)
                ctx.set_stream(self.stream.cuda_stream)
                ctx._shard_step_stream = self.stream
        else:
            self.stream = _HostStream()
        self.rows_seen = False  # some rank had rows in the last finished step
        self._no_rows = None
        # the gathered counts go to pinned host memory by an async copy queued
        # behind the all_gather; finish() waits on its event and reads them (no
        # synchronous device-to-host read per step: the host's share of a short
        # step, e.g. one of eight shards of config 4)
        self.pinned = device.type == "cuda" and not self.host and counts is None
        if self.pinned:
            self.cnts_host = torch.empty(world, dtype=torch.int64, pin_memory=True)
            self.cnts_evt = torch.cuda.Event()

    def enqueue(self, thr, chunk_begin, chunk_end, kernel_done=None):
        """The pair kernel, its row count and the count all_gather, on the
        context's stream; no host wait.  kernel_done (a torch.cuda.Event) is
        recorded after the kernel, before the collective."""
        import torch
        import torch.distributed as dist

        g = self.gather
        if self.xchg is not None:  # the pass alone: its count is read on the host in finish()
            self.ctx.run_chunks_async(thr, chunk_begin, chunk_end)
            if kernel_done is not None:
                kernel_done.record(self.stream)
            return
        with _stream_scope(self.stream):
            self.ctx.run_chunks_async(thr, chunk_begin, chunk_end, (self.cnt_dev if self.host else g.cnt).data_ptr())
            if kernel_done is not None:
                kernel_done.record(self.stream)
            if not self.host:
                dist.all_gather_into_tensor(g.cnts, g.cnt, group=g.group)
                if self.pinned:
                    self.cnts_host.copy_(g.cnts, non_blocking=True)
                    self.cnts_evt.record(self.stream)

    def finish(self):
        """Completes an enqueued step: (rows on this rank, gathered rows on rank 0 / None)."""
        import torch
        import torch.distributed as dist

        g = self.gather
        if self.xchg is not None:
            n = self.ctx.run_wait()  # this rank's pass completed; its row count on the host
            counts = self.xchg(n)
            self.rows_seen = max(counts) > 0
            if not self.rows_seen:
                if self._no_rows is None:
                    self._no_rows = g.cnt.new_zeros((5, 0), dtype=torch.int32)
                return n, (self._no_rows if g.rank == 0 else None)
            packed = pack_rows_device(self.ctx, n, self.device)
            if self.host:
                packed = packed.cpu()
            return n, (packed if g.world == 1 else g(packed, counts))
        if self.host:
            with _stream_scope(self.stream):
                g.cnt.fill_(int(self.cnt_dev.item()))  # host wait for this step's count
            dist.all_gather_into_tensor(g.cnts, g.cnt, group=g.group)
        if self.pinned:
            self.cnts_evt.synchronize()  # the step's one host wait when no rank has rows
            counts = self.cnts_host.tolist()
        else:
            with _stream_scope(self.stream):
                counts = g.cnts.tolist()  # the step's one host wait when no rank has rows
        self.rows_seen = max(counts) > 0
        n = self.ctx.run_wait()  # returns at once: the stream is idle
        if max(counts) == 0:
            if self._no_rows is None:  # (one empty result, not an allocation per step)
                self._no_rows = g.cnt.new_zeros((5, 0), dtype=torch.int32)
            return n, (self._no_rows if g.rank == 0 else None)
        packed = pack_rows_device(self.ctx, n, self.device)
        if self.host:
            packed = packed.cpu()
        return n, (packed if g.world == 1 else g(packed, counts))

    def __call__(self, thr, chunk_begin, chunk_end):
        self.enqueue(thr, chunk_begin, chunk_end)
        return self.finish()

    def close(self):
        """Waits for the step's stream; the context keeps running on it until
        its owner closes it (its buffers are freed after that stream's work)."""
        if not isinstance(self.stream, _HostStream):
            self.stream.synchronize()


class PipelinedShardStep:
    """Back-to-back ShardSteps on D >= 2 contexts loaded with the same inputs
    (D-buffered staging and counts).  Step i runs on context i % D and up to
    D - 1 steps are in flight: submit() enqueues step i, then completes the
    oldest step once more than D - 1 are pending, so that step's count
    exchange, host read and (if any rank has rows) row gather overlap the
    kernels queued behind it.  serialize_kernels=False lets step i's kernel
    start in the tail of step i-1's (the contexts share nothing the kernels
    write); True makes it wait on the device (an event, no host wait) for
    step i-1's whole run (pair kernels, row count, count all_gather); "pair"
    only for step i-1's pair kernel (wld_run_after: the small kernels after
    it overlap step i's), so pair kernels run one at a time with the next
    already queued.  The full wait is also done while the last finished step
    had rows, so a step's row copies and gather do not compete with two
    kernels.  submit() returns the
    completed step's result (None while the pipeline fills); drain_all()
    completes the pending steps and returns their results in step order,
    drain() the last of them (or None).  Collectives are issued in step order
    on every rank (count all_gathers in submit order, a step's row gather when
    it completes), so the sequence is the same everywhere."""

    def __init__(self, ctxs, rank, world, device, group=None, serialize_kernels=False, host_collectives=False,
                 counts=None):
        import torch

        assert len(ctxs) >= 2
        self.steps = [ShardStep(c, rank, world, device, group, host_collectives, counts) for c in ctxs]
        self.done = ([torch.cuda.Event() for _ in ctxs] if torch.device(device).type == "cuda"
                     else [_HostEvent() for _ in ctxs])
        self.serialize = serialize_kernels  # False: step i's kernel may start in step i-1's tail
        self.i = 0
        self.pending = collections.deque()  # contexts of the enqueued, unfinished steps, oldest first
        self.recorded = [False] * len(ctxs)  # done[k] recorded after context k's latest enqueued step

    def submit(self, thr, chunk_begin, chunk_end):
        D = len(self.steps)
        k = self.i % D
        assert k not in self.pending  # step i - D completed in an earlier submit
        if self.pending:
            prev = self.pending[-1]
            if any(st.rows_seen for st in self.steps) or (self.serialize and self.serialize != "pair"):
                if not self.recorded[prev]:
                    # prev was enqueued without its end event (no rank had
                    # rows then); nothing has been queued on its stream since,
                    # so a record now marks exactly the end of prev's step
                    self.done[prev].record(self.steps[prev].stream)
                    self.recorded[prev] = True
                self.steps[k].stream.wait_event(self.done[prev])
            elif self.serialize == "pair":
                self.steps[k].ctx.run_after(self.steps[prev].ctx)
        # the step's end event only where a later submit may wait on it (a
        # wait_event on an older record of the same event only orders less:
        # the contexts share nothing the kernels write); one record fewer per
        # step in the common case
        need_done = self.serialize is True or any(st.rows_seen for st in self.steps)
        self.steps[k].enqueue(thr, chunk_begin, chunk_end, self.done[k] if need_done else None)
        self.recorded[k] = need_done
        self.i += 1
        self.pending.append(k)
        return self.steps[self.pending.popleft()].finish() if len(self.pending) > D - 1 else None

    def drain_all(self):
        out = []
        while self.pending:
            out.append(self.steps[self.pending.popleft()].finish())
        return out

    def drain(self):
        out = self.drain_all()
        return out[-1] if out else None

    def close(self):
        self.drain_all()
        for st in self.steps:
            st.close()


def gather_rows(packed, rank, world, group=None):
    """One-shot RowGather: every rank's [5, n_r] rows to rank 0 in reference
    order (shards in descending rank order), None elsewhere."""
    return RowGather(rank, world, packed.device, group)(packed)
