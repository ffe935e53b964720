"""Python mirror of the weighted_ld crate's public surface (rust/weighted_ld/src/lib.rs).

Same names, argument meaning and results as the Rust functions, implemented on
the C ABI of libweightedld.so: the host pre-pass (FASTA, site filter, Henikoff
weights) runs in the library's C++ host code, the all-pairs hot path on the
gfx950 GPU.  There is no CPU fallback for the hot path.
"""
import atexit
import ctypes
import weakref
import enum
from collections import namedtuple

import numpy as np

from ._lib import (KERNEL_AUTO, KERNEL_MFMA, KERNEL_VALU, OPTIONS, PROGRESS_FN, Pairs, RunStats, WldError, check,
                   lib)

__all__ = [
    "Symbol", "SymbolHistogram", "SiteSet", "LdStats", "PairStore", "read_fasta", "read_vcf",
    "is_site_of_interest", "henikoff_weights", "single_weighted_ld_pair", "all_weighted_ld_pairs",
    "Context", "default_context", "KERNEL_AUTO", "KERNEL_VALU", "KERNEL_MFMA", "OPTIONS", "WldError",
]


def _p(a, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct))


class Symbol(enum.IntEnum):
    """lib.rs:20-29 (#[repr(u8)])."""
    A = 0
    C = 1
    G = 2
    T = 3
    Missing = 4
    Unknown = 5

    @staticmethod
    def from_char(c):
        """lib.rs:53-64."""
        return {"a": Symbol.A, "A": Symbol.A, "c": Symbol.C, "C": Symbol.C, "g": Symbol.G, "G": Symbol.G,
                "t": Symbol.T, "T": Symbol.T, "-": Symbol.Missing}.get(c, Symbol.Unknown)

    def is_acgt(self):
        return self <= Symbol.T

    def is_acgtm(self):
        return self <= Symbol.Missing


def symbols_from_str(s):
    return np.array([Symbol.from_char(c) for c in s], dtype=np.uint8)


class SymbolHistogram:
    """lib.rs:72-141."""

    def __init__(self, counts):
        self.data = np.asarray(counts, dtype=np.uint64).reshape(6)

    @staticmethod
    def from_slice(symbols):
        s = np.ascontiguousarray(symbols, dtype=np.uint8)
        h = np.zeros(6, dtype=np.uint64)
        check(lib().wld_histogram(_p(s, ctypes.c_uint8), s.size, _p(h, ctypes.c_uint64)), "histogram")
        return SymbolHistogram(h)

    def __getitem__(self, sym):
        return int(self.data[int(sym)])

    def major_minor_symbols(self):
        a, b = ctypes.c_int(), ctypes.c_int()
        h = np.ascontiguousarray(self.data)
        check(lib().wld_major_minor(_p(h, ctypes.c_uint64), ctypes.byref(a), ctypes.byref(b)), "major_minor")
        return (Symbol(a.value) if a.value >= 0 else None, Symbol(b.value) if b.value >= 0 else None)


class SiteSet:
    """lib.rs:158-275: site-major symbol buffer, optional site_map, histograms."""

    def __init__(self, handle):
        self._h = ctypes.c_void_p(handle)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and lib is not None:
            try:
                lib().wld_siteset_free(h)
            except Exception:
                pass
            self._h = None

    @staticmethod
    def from_buffer(site_major, site_map=None):
        """Builds a SiteSet from a [n_sites, n_seqs] uint8 array of Symbol codes."""
        buf = np.ascontiguousarray(site_major, dtype=np.uint8)
        if buf.ndim != 2:
            raise ValueError("site_major must be [n_sites, n_seqs]")
        sm = None if site_map is None else np.ascontiguousarray(site_map, dtype=np.uint64)
        out = ctypes.c_void_p()
        check(lib().wld_siteset_from_buffer(_p(buf, ctypes.c_uint8), buf.shape[0], buf.shape[1],
                                            None if sm is None else _p(sm, ctypes.c_uint64), ctypes.byref(out)),
              "siteset_from_buffer")
        return SiteSet(out.value)

    @staticmethod
    def from_strs(seqs):
        """lib.rs:208-228 (test helper): one string per sequence."""
        return SiteSet.from_buffer(np.stack([symbols_from_str(s) for s in seqs], axis=1))

    def n_sites(self):
        return lib().wld_siteset_n_sites(self._h)

    def n_seqs(self):
        return lib().wld_siteset_n_seqs(self._h)

    @property
    def buffer(self):
        """SiteSet.buffer as a [n_sites, n_seqs] uint8 array (copy)."""
        L, N = self.n_sites(), self.n_seqs()
        if L * N == 0:
            return np.zeros((L, N), dtype=np.uint8)
        p = lib().wld_siteset_buffer(self._h)
        return np.ctypeslib.as_array(p, shape=(L * N,)).reshape(L, N).copy()

    @property
    def site_map(self):
        p = lib().wld_siteset_site_map(self._h)
        if not p:
            return None
        return np.ctypeslib.as_array(p, shape=(self.n_sites(),)).copy()

    def parent_site_index(self, idx):
        return int(lib().wld_siteset_parent_site_index(self._h, idx))

    def site_symbols(self, index):
        return self.buffer[index]

    def site_histogram(self, index):
        h = np.zeros(6, dtype=np.uint64)
        check(lib().wld_siteset_histogram(self._h, index, _p(h, ctypes.c_uint64)), "site_histogram")
        return SymbolHistogram(h)

    def filter_sites_of_interest(self, min_acgt=0.8, min_minor=0.02, max_minor=0.5):
        """main.rs:139-143: filter_by(|s| is_site_of_interest(s, ceil(min_acgt*N), min_minor, max_minor))."""
        out = ctypes.c_void_p()
        check(lib().wld_siteset_filter_sites_of_interest(self._h, min_acgt, min_minor, max_minor,
                                                         ctypes.byref(out)), "filter_by")
        return SiteSet(out.value)


def read_fasta(path):
    """read_fasta + SiteSet::from_multiseq (lib.rs:277-307, 176-206)."""
    out = ctypes.c_void_p()
    check(lib().wld_read_fasta(str(path).encode(), ctypes.byref(out)), "read_fasta")
    return SiteSet(out.value)


def read_vcf(path):
    """VCF reader with WeightedLD.py handle_vcf semantics (WeightedLD.py:311-379)."""
    out = ctypes.c_void_p()
    check(lib().wld_read_vcf(str(path).encode(), ctypes.byref(out)), "read_vcf")
    return SiteSet(out.value)


def is_site_of_interest(site, min_acgt, min_minor, max_minor):
    """lib.rs:309-338 (min_acgt is a count)."""
    s = np.ascontiguousarray(site, dtype=np.uint8)
    return bool(lib().wld_is_site_of_interest(_p(s, ctypes.c_uint8), s.size, int(min_acgt), min_minor, max_minor))


def henikoff_weights(site_set):
    """lib.rs:340-380."""
    w = np.zeros(site_set.n_seqs(), dtype=np.float32)
    check(lib().wld_henikoff_weights(site_set._h, _p(w, ctypes.c_float)), "henikoff_weights")
    return w


LdStats = namedtuple("LdStats", ["r2", "d", "d_prime"])  # lib.rs:382-387


class PairStore:
    """PairStore<LdStats> (lib.rs:529-576) as structure-of-arrays in reference order."""

    def __init__(self, site_a, site_b, d, d_prime, r2):
        self.site_a, self.site_b, self.d, self.d_prime, self.r2 = site_a, site_b, d, d_prime, r2

    def __len__(self):
        return int(self.site_a.size)

    def len(self):
        return len(self)

    def iter(self):
        for i in range(len(self)):
            yield (int(self.site_a[i]), int(self.site_b[i]),
                   LdStats(float(self.r2[i]), float(self.d[i]), float(self.d_prime[i])))

    __iter__ = iter


# Live contexts, closed (newest first) by an exit handler while the HIP
# runtime and torch are still up: a context left to its finalizer at
# interpreter shutdown would destroy its stream and buffers in arbitrary order
# against torch objects that may still reference them (events, pinned-memory
# copies recorded on a stream the context ran on).
_LIVE = weakref.WeakValueDictionary()
_SEQ = [0]


@atexit.register
def _close_live_contexts():
    for k in sorted(list(_LIVE.keys()), reverse=True):
        c = _LIVE.get(k)
        if c is not None:
            try:
                c.close()
            except Exception:
                pass


class Context:
    """One device context (wld_ctx): HIP stream, device buffers, results."""

    def __init__(self, device=0, kernel=KERNEL_AUTO, devices=None, ref_sums=None):
        """devices (a list of HIP ordinals, repeats allowed): a multi-device
        context (wld_create_multi) that shards load/run_host/all-pairs calls.
        ref_sums (WLD_OPT_REF_SUMS): None keeps the library default (lib.rs's
        own f32 summation order, bit-identical rows); False: exact sums."""
        self._borrowers = weakref.WeakSet()  # contexts running on this one's stream (set_stream)
        self._stream_owner = None
        h = ctypes.c_void_p()
        self._lib = lib()  # kept: module globals may be gone when __del__ runs at exit
        if devices is not None:
            arr = (ctypes.c_int * len(devices))(*devices)
            check(self._lib.wld_create_multi(arr, len(devices), ctypes.byref(h)), "wld_create_multi")
            device = devices[0]
        else:
            check(self._lib.wld_create(device, ctypes.byref(h)), "wld_create")
        self._h = h
        self.device = device
        _SEQ[0] += 1
        _LIVE[_SEQ[0]] = self
        if kernel != KERNEL_AUTO:
            self.set_kernel(kernel)
        if ref_sums is not None:
            self.set_option("ref_sums", int(bool(ref_sums)))

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            # contexts running on this one's stream get their own back first
            # (wld_set_stream waits for their queued work)
            for b in list(getattr(self, "_borrowers", ())):
                if getattr(b, "_h", None) is not None and b._h.value:
                    b.set_stream(None)
            owner = getattr(self, "_stream_owner", None)
            if owner is not None:
                owner._borrowers.discard(self)
                self._stream_owner = None
            self._lib.wld_destroy(self._h)
            self._h = None

    __del__ = close

    def n_devices(self):
        return int(lib().wld_n_devices(self._h))

    def set_kernel(self, kernel):
        check(lib().wld_set_kernel(self._h, kernel), "wld_set_kernel")

    def set_option(self, name, value):
        """wld_set_option: name is a key of OPTIONS ("prefilter", "screen",
        "tile_order", "all_planes", "mfma_layout", "valu_plain", "staging_rows",
        "host_batch_pairs", "ref_sums", "fused_scan"); only "ref_sums" changes a result."""
        check(lib().wld_set_option(self._h, OPTIONS[name], int(value)), "wld_set_option")

    def get_option(self, name):
        v = ctypes.c_int64()
        check(lib().wld_get_option(self._h, OPTIONS[name], ctypes.byref(v)), "wld_get_option")
        return int(v.value)

    def load(self, site_major, weights, site_map=None):
        buf = np.ascontiguousarray(site_major, dtype=np.uint8)
        w = np.ascontiguousarray(weights, dtype=np.float32)
        if buf.ndim != 2 or w.size != buf.shape[1]:
            raise ValueError("site_major must be [n_sites, n_seqs] and weights n_seqs long")
        sm = None if site_map is None else np.ascontiguousarray(site_map, dtype=np.uint64)
        check(lib().wld_load(self._h, _p(buf, ctypes.c_uint8), buf.shape[0], buf.shape[1],
                             None if sm is None else _p(sm, ctypes.c_uint64), _p(w, ctypes.c_float)), "wld_load")

    def load_device(self, d_sites_ptr, n_sites, n_seqs, d_weights_ptr, site_map=None):
        sm = None if site_map is None else np.ascontiguousarray(site_map, dtype=np.uint64)
        check(lib().wld_load_device(self._h, ctypes.c_void_p(d_sites_ptr), n_sites, n_seqs,
                                    None if sm is None else _p(sm, ctypes.c_uint64),
                                    ctypes.c_void_p(d_weights_ptr)), "wld_load_device")

    def load_filtered(self, buffer, min_acgt=0.8, min_minor=0.02, max_minor=0.5, unweighted=False, site_map=None):
        """Device pre-pass (main.rs:139-156 on the GPU): filter the UNFILTERED
        [n_sites, n_seqs] Symbol buffer with is_site_of_interest, compute
        Henikoff (or unit) weights on the kept sites and load them.  Returns the
        kept site count; weights() and site_map() give the pre-pass results."""
        buf = np.ascontiguousarray(buffer, dtype=np.uint8)
        L, N = buf.shape
        sm = None if site_map is None else np.ascontiguousarray(site_map, dtype=np.uint64)
        n = ctypes.c_size_t()
        check(lib().wld_load_filtered(self._h, _p(buf, ctypes.c_uint8), L, N,
                                      None if sm is None else _p(sm, ctypes.c_uint64), min_acgt, min_minor, max_minor,
                                      int(bool(unweighted)), ctypes.byref(n)), "wld_load_filtered")
        self._n_seqs, self._n_kept = N, int(n.value)
        return self._n_kept

    def load_filtered_device(self, d_sites_ptr, n_sites, n_seqs, min_acgt=0.8, min_minor=0.02, max_minor=0.5,
                             unweighted=False, site_map=None):
        sm = None if site_map is None else np.ascontiguousarray(site_map, dtype=np.uint64)
        n = ctypes.c_size_t()
        check(lib().wld_load_filtered_device(self._h, ctypes.c_void_p(d_sites_ptr), n_sites, n_seqs,
                                             None if sm is None else _p(sm, ctypes.c_uint64), min_acgt,
                                             min_minor, max_minor, int(bool(unweighted)), ctypes.byref(n)),
              "wld_load_filtered_device")
        self._n_seqs, self._n_kept = n_seqs, int(n.value)
        return self._n_kept

    def weights(self):
        w = np.zeros(self._n_seqs, dtype=np.float32)
        check(lib().wld_weights_copy(self._h, _p(w, ctypes.c_float)), "wld_weights_copy")
        return w

    def site_map(self):
        m = np.zeros(self._n_kept, dtype=np.uint64)
        check(lib().wld_site_map_copy(self._h, _p(m, ctypes.c_uint64)), "wld_site_map_copy")
        return m

    def run(self, r2_threshold, row_begin=0, row_end=0):
        n = ctypes.c_uint64()
        check(lib().wld_run(self._h, r2_threshold, row_begin, row_end, ctypes.byref(n)), "wld_run")
        return int(n.value)

    def run_chunks(self, r2_threshold, chunk_begin=0, chunk_end=0):
        """wld_run_chunks: pairs of the linear chunk range [chunk_begin, chunk_end) (end 0 = all)."""
        n = ctypes.c_uint64()
        check(lib().wld_run_chunks(self._h, r2_threshold, chunk_begin, chunk_end, ctypes.byref(n)), "wld_run_chunks")
        return int(n.value)

    def run_chunks_async(self, r2_threshold, chunk_begin=0, chunk_end=0, d_count_ptr=None):
        """wld_run_chunks_async: enqueue the run on the context's stream; the row
        total lands in the device uint64 at d_count_ptr (if given).  Complete
        it with run_wait() before any other call on this context."""
        check(lib().wld_run_chunks_async(self._h, r2_threshold, chunk_begin, chunk_end,
                                         ctypes.c_void_p(d_count_ptr) if d_count_ptr else None),
              "wld_run_chunks_async")

    def run_wait(self):
        """wld_run_wait: completes the run started by run_chunks_async; returns its row count."""
        n = ctypes.c_uint64()
        check(lib().wld_run_wait(self._h, ctypes.byref(n)), "wld_run_wait")
        return int(n.value)

    def run_after(self, prev):
        """wld_run_after: this context's next run waits on the device for the
        pair kernels of prev's run in flight (no host wait)."""
        check(lib().wld_run_after(self._h, prev._h), "wld_run_after")

    def run_host(self, r2_threshold, progress_report=None):
        """wld_run_host: every pair of the loaded set, in batches of <= 2^31
        pairs, rows to host in reference order (a PairStore)."""
        cb = PROGRESS_FN(lambda n, _u: progress_report(int(n))) if progress_report else PROGRESS_FN()
        out = Pairs()
        check(lib().wld_run_host(self._h, r2_threshold, cb, None, ctypes.byref(out)), "wld_run_host")
        return _take_pairs(out)

    def stream_ptr(self):
        """The context's hipStream_t as an int (torch.cuda.ExternalStream)."""
        return int(lib().wld_stream(self._h) or 0)

    def set_stream(self, stream):
        """wld_set_stream: run on another context's stream (a Context), a
        hipStream_t given as an int, or None for the context's own.  A borrowed
        Context stream stays referenced here, and the owner hands this context
        back its own stream before its close() destroys the borrowed one."""
        ptr = stream.stream_ptr() if isinstance(stream, Context) else (stream or 0)
        check(lib().wld_set_stream(self._h, ctypes.c_void_p(ptr) if ptr else None), "wld_set_stream")
        old = getattr(self, "_stream_owner", None)
        if old is not None:
            old._borrowers.discard(self)
        self._stream_owner = stream if isinstance(stream, Context) else None
        if self._stream_owner is not None:
            self._stream_owner._borrowers.add(self)

    def rows(self):
        v = Pairs()
        check(lib().wld_rows_device(self._h, ctypes.byref(v)), "wld_rows_device")
        n = int(v.n)
        a = np.zeros(n, dtype=np.uint32)
        b = np.zeros(n, dtype=np.uint32)
        d = np.zeros(n, dtype=np.float32)
        dp = np.zeros(n, dtype=np.float32)
        r2 = np.zeros(n, dtype=np.float32)
        if n:
            check(lib().wld_rows_copy(self._h, _p(a, ctypes.c_uint32), _p(b, ctypes.c_uint32), _p(d, ctypes.c_float),
                                      _p(dp, ctypes.c_float), _p(r2, ctypes.c_float)), "wld_rows_copy")
        return PairStore(a, b, d, dp, r2)

    def rows_device(self):
        v = Pairs()
        check(lib().wld_rows_device(self._h, ctypes.byref(v)), "wld_rows_device")
        addr = lambda p: ctypes.cast(p, ctypes.c_void_p).value or 0  # noqa: E731
        return {"n": int(v.n), "site_a": addr(v.site_a), "site_b": addr(v.site_b), "d": addr(v.d),
                "d_prime": addr(v.d_prime), "r2": addr(v.r2)}

    def rows_copy_device(self, site_a, site_b, d, d_prime, r2):
        """Copies the last run's rows into caller device buffers (raw pointers, 0 = skip)."""
        vp = lambda x: ctypes.c_void_p(x or None)  # noqa: E731
        check(lib().wld_rows_copy_device(self._h, vp(site_a), vp(site_b), vp(d), vp(d_prime), vp(r2)),
              "wld_rows_copy_device")

    def dense(self, n_sites):
        d = np.zeros((n_sites, n_sites), dtype=np.float32)
        dp = np.zeros_like(d)
        r2 = np.zeros_like(d)
        valid = np.zeros((n_sites, n_sites), dtype=np.uint8)
        check(lib().wld_dense(self._h, _p(d, ctypes.c_float), _p(dp, ctypes.c_float), _p(r2, ctypes.c_float),
                              _p(valid, ctypes.c_uint8)), "wld_dense")
        return d, dp, r2, valid

    def stats(self):
        s = RunStats()
        check(lib().wld_last_stats(self._h, ctypes.byref(s)), "wld_last_stats")
        return {f: getattr(s, f) for f, _ in RunStats._fields_}

    @staticmethod
    def chunk_rows(n_sites):
        return int(lib().wld_chunk_rows(n_sites))

    @staticmethod
    def shard_chunk_rows(n_sites, n_shards, shard):
        b, e = ctypes.c_uint32(), ctypes.c_uint32()
        check(lib().wld_shard_chunk_rows(n_sites, n_shards, shard, ctypes.byref(b), ctypes.byref(e)), "shard")
        return int(b.value), int(e.value)

    @staticmethod
    def chunks(n_sites):
        return int(lib().wld_chunks(n_sites))

    @staticmethod
    def shard_chunks(n_sites, n_shards, shard):
        """Linear chunk range [begin, end) of `shard` (wld_shard_chunks)."""
        b, e = ctypes.c_uint32(), ctypes.c_uint32()
        check(lib().wld_shard_chunks(n_sites, n_shards, shard, ctypes.byref(b), ctypes.byref(e)), "shard_chunks")
        return int(b.value), int(e.value)

    @staticmethod
    def pairs_in_chunks(n_sites, begin, end):
        return int(lib().wld_pairs_in_chunks(n_sites, begin, end))


_default = {}


def default_context(device=0):
    if device not in _default:
        _default[device] = Context(device)
    return _default[device]


def single_weighted_ld_pair(a, a_hist, b, b_hist, weights, ctx=None):
    """lib.rs:390-521 -> LdStats or None.  a_hist/b_hist are accepted for
    signature parity; the device derives the same histograms from a and b."""
    ctx = ctx or default_context()
    av = np.ascontiguousarray(a, dtype=np.uint8)
    bv = np.ascontiguousarray(b, dtype=np.uint8)
    w = np.ascontiguousarray(weights, dtype=np.float32)
    if not (av.size == bv.size == w.size):
        raise ValueError("a, b and weights must have the same length (lib.rs:397-398)")
    out = np.zeros(3, dtype=np.float32)
    r = check(lib().wld_single_weighted_ld_pair(ctx._h, _p(av, ctypes.c_uint8), _p(bv, ctypes.c_uint8),
                                                _p(w, ctypes.c_float), av.size, _p(out, ctypes.c_float)),
              "single_weighted_ld_pair")
    if r == 0:
        return None
    return LdStats(r2=float(out[2]), d=float(out[0]), d_prime=float(out[1]))


def all_weighted_ld_pairs(site_set, weights, r2_threshold, progress_report=None, ctx=None):
    """lib.rs:578-684 -> PairStore in reference order (parent site indices)."""
    ctx = ctx or default_context()
    buf = site_set.buffer
    w = np.ascontiguousarray(weights, dtype=np.float32)
    if w.size != site_set.n_seqs():
        raise ValueError("weights must have n_seqs entries")
    sm = site_set.site_map
    cb = PROGRESS_FN(lambda n, _u: progress_report(int(n))) if progress_report else PROGRESS_FN()
    out = Pairs()
    check(lib().wld_all_weighted_ld_pairs(ctx._h, _p(buf, ctypes.c_uint8), buf.shape[0], buf.shape[1],
                                          None if sm is None else _p(sm, ctypes.c_uint64), _p(w, ctypes.c_float),
                                          r2_threshold, cb, None, ctypes.byref(out)), "all_weighted_ld_pairs")
    return _take_pairs(out)


def _take_pairs(out):
    """Library-allocated host wld_pairs -> PairStore (copies, then frees)."""
    n = int(out.n)

    def grab(p, dt):
        return np.ctypeslib.as_array(p, shape=(n,)).astype(dt, copy=True) if n else np.zeros(0, dtype=dt)

    store = PairStore(grab(out.site_a, np.uint32), grab(out.site_b, np.uint32), grab(out.d, np.float32),
                      grab(out.d_prime, np.float32), grab(out.r2, np.float32))
    lib().wld_pairs_free(ctypes.byref(out))
    return store
