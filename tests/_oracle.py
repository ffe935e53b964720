"""ctypes loader for the CPU oracle (oracle/wld_oracle.c).

TEST INFRASTRUCTURE: imported only by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py — never by the product package.
"""
import ctypes
import hashlib
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "libwld_oracle.so")


class _Rows(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint64),
        ("site_a", ctypes.POINTER(ctypes.c_uint64)),
        ("site_b", ctypes.POINTER(ctypes.c_uint64)),
        ("d", ctypes.POINTER(ctypes.c_float)),
        ("d_prime", ctypes.POINTER(ctypes.c_float)),
        ("r2", ctypes.POINTER(ctypes.c_float)),
    ]


_lib = None


def use_native():
    """Builds the oracle for THIS host (-march=native, into oracle/build_native)
    and makes lib() load that build: bench.py's CPU baseline, on the measuring
    host (the test build is -march=x86-64-v3 so it runs on any x86-64 host)."""
    global ORACLE_SO, _lib
    out = os.path.join(ORACLE_DIR, "build_native")
    subprocess.run(["make", "-s", "-B", "-C", ORACLE_DIR, "MARCH=native", "OUT=" + out], check=True)
    ORACLE_SO = os.path.join(out, "libwld_oracle.so")
    _lib = None
    return ORACLE_SO


def lib():
    global _lib
    if _lib is not None:
        return _lib
    src = os.path.join(ORACLE_DIR, "wld_oracle.c")
    if not os.path.exists(ORACLE_SO) or os.path.getmtime(ORACLE_SO) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    L = ctypes.CDLL(ORACLE_SO)
    u8p = ctypes.POINTER(ctypes.c_uint8)
    u64p = ctypes.POINTER(ctypes.c_uint64)
    f32p = ctypes.POINTER(ctypes.c_float)
    sz = ctypes.c_size_t
    L.wldo_read_fasta.argtypes = [ctypes.c_char_p, ctypes.POINTER(u8p), ctypes.POINTER(sz), ctypes.POINTER(sz)]
    L.wldo_read_fasta.restype = ctypes.c_int
    L.wldo_free.argtypes = [ctypes.c_void_p]
    L.wldo_histogram.argtypes = [u8p, sz, u64p]
    L.wldo_major_minor.argtypes = [u64p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    L.wldo_is_site_of_interest.argtypes = [u8p, sz, sz, ctypes.c_float, ctypes.c_float]
    L.wldo_is_site_of_interest.restype = ctypes.c_int
    L.wldo_min_acgt_count.argtypes = [ctypes.c_float, sz]
    L.wldo_min_acgt_count.restype = sz
    L.wldo_henikoff_weights.argtypes = [u8p, sz, sz, f32p]
    L.wldo_single_pair.argtypes = [u8p, u8p, f32p, sz, f32p]
    L.wldo_single_pair.restype = ctypes.c_int
    L.wldo_all_pairs_range.argtypes = [u8p, sz, sz, u64p, f32p, ctypes.c_float, ctypes.c_int, sz, sz,
                                       ctypes.POINTER(_Rows)]
    L.wldo_all_pairs_range.restype = ctypes.c_int64
    L.wldo_rows_free.argtypes = [ctypes.POINTER(_Rows)]
    L.wldo_all_pairs_dense.argtypes = [u8p, sz, sz, f32p, f32p, f32p, f32p, u8p]
    L.wldo_triu_index.argtypes = [sz, sz, ctypes.POINTER(sz), ctypes.POINTER(sz)]
    f64p = ctypes.POINTER(ctypes.c_double)
    L.wldo_all_pairs_dense_f64.argtypes = [u8p, sz, sz, f32p, f64p, f64p, f64p, u8p]
    L.wldo_set_hsum_order.argtypes = [ctypes.c_int]
    L.wldo_get_hsum_order.restype = ctypes.c_int
    _lib = L
    return L


class hsum_order:
    """Context manager selecting the f32x8 horizontal-sum order of the oracle's
    lane sums (lib.rs:447-452): "ordered" (((0+x0)+x1)+...+x7, packed_simd's
    x86 implementation, the default) or "tree" (its documented order)."""

    def __init__(self, order):
        self.tree = {"ordered": 0, "tree": 1}[order]

    def __enter__(self):
        self.prev = lib().wldo_get_hsum_order()
        lib().wldo_set_hsum_order(self.tree)
        return self

    def __exit__(self, *exc):
        lib().wldo_set_hsum_order(self.prev)


def _p(arr, ct):
    return arr.ctypes.data_as(ctypes.POINTER(ct))


def symbols(s):
    """lib.rs:53-64 on a str (test helper)."""
    L = lib()
    return np.array([L.wldo_symbol_from_char(ord(c)) for c in s], dtype=np.uint8)


def read_fasta(path):
    """Returns (buffer[n_sites, n_seqs] uint8 site-major, n_seqs, n_sites) or raises."""
    L = lib()
    buf = ctypes.POINTER(ctypes.c_uint8)()
    ns, nl = ctypes.c_size_t(), ctypes.c_size_t()
    rc = L.wldo_read_fasta(path.encode(), ctypes.byref(buf), ctypes.byref(ns), ctypes.byref(nl))
    if rc == -1:
        raise OSError(path)
    if rc == -2:
        raise ValueError("Not all sequences have the same number of symbols")
    n = ns.value * nl.value
    out = np.ctypeslib.as_array(buf, shape=(max(n, 1),))[:n].copy().reshape(nl.value, ns.value)
    L.wldo_free(buf)
    return out


def histogram(site):
    site = np.ascontiguousarray(site, dtype=np.uint8)
    h = np.zeros(6, dtype=np.uint64)
    lib().wldo_histogram(_p(site, ctypes.c_uint8), site.size, _p(h, ctypes.c_uint64))
    return h


def major_minor(hist):
    h = np.ascontiguousarray(hist, dtype=np.uint64)
    a, b = ctypes.c_int(), ctypes.c_int()
    lib().wldo_major_minor(_p(h, ctypes.c_uint64), ctypes.byref(a), ctypes.byref(b))
    return (a.value if a.value >= 0 else None, b.value if b.value >= 0 else None)


def site_mask(buf, min_acgt=0.8, min_minor=0.02, max_minor=0.5):
    """main.rs:139-143 → boolean mask over sites."""
    L = lib()
    n_sites, n_seqs = buf.shape
    thr = L.wldo_min_acgt_count(min_acgt, n_seqs)
    buf = np.ascontiguousarray(buf)
    return np.array([bool(L.wldo_is_site_of_interest(_p(buf[s], ctypes.c_uint8), n_seqs, thr,
                                                      min_minor, max_minor)) for s in range(n_sites)])


def henikoff_weights(buf):
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    n_sites, n_seqs = buf.shape
    w = np.zeros(n_seqs, dtype=np.float32)
    lib().wldo_henikoff_weights(_p(buf, ctypes.c_uint8), n_sites, n_seqs, _p(w, ctypes.c_float))
    return w


def single_pair(a, b, w):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    b = np.ascontiguousarray(b, dtype=np.uint8)
    w = np.ascontiguousarray(w, dtype=np.float32)
    out = np.zeros(3, dtype=np.float32)
    ok = lib().wldo_single_pair(_p(a, ctypes.c_uint8), _p(b, ctypes.c_uint8), _p(w, ctypes.c_float),
                                a.size, _p(out, ctypes.c_float))
    return (float(out[0]), float(out[1]), float(out[2])) if ok else None


def all_pairs(buf, weights, thr, site_map=None, n_threads=None, chunk_lo=0, chunk_hi=None):
    """lib.rs:578-684 → dict of numpy arrays in reference (triu chunk) order, plus pair count."""
    L = lib()
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    n_sites, n_seqs = buf.shape
    w = np.ascontiguousarray(weights, dtype=np.float32)
    sm = None if site_map is None else np.ascontiguousarray(site_map, dtype=np.uint64)
    rows = _Rows()
    # OMP_NUM_THREADS: the GPU box's CPU share (16) when cpu_count() shows the whole machine
    nt = n_threads or int(os.environ.get("OMP_NUM_THREADS") or 0) or (os.cpu_count() or 1)
    hi = ctypes.c_size_t(-1).value if chunk_hi is None else chunk_hi
    n = L.wldo_all_pairs_range(_p(buf, ctypes.c_uint8), n_sites, n_seqs,
                               None if sm is None else _p(sm, ctypes.c_uint64), _p(w, ctypes.c_float),
                               thr, nt, chunk_lo, hi, ctypes.byref(rows))
    k = rows.n

    def grab(ptr, dt):
        if k == 0:
            return np.zeros(0, dtype=dt)
        return np.ctypeslib.as_array(ptr, shape=(k,)).copy()

    out = {"site_a": grab(rows.site_a, np.uint64), "site_b": grab(rows.site_b, np.uint64),
           "d": grab(rows.d, np.float32), "d_prime": grab(rows.d_prime, np.float32),
           "r2": grab(rows.r2, np.float32), "pairs": int(n)}
    L.wldo_rows_free(ctypes.byref(rows))
    return out


def all_pairs_dense(buf, weights):
    L = lib()
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    n_sites, n_seqs = buf.shape
    w = np.ascontiguousarray(weights, dtype=np.float32)
    d = np.zeros((n_sites, n_sites), dtype=np.float32)
    dp = np.zeros_like(d)
    r2 = np.zeros_like(d)
    valid = np.zeros((n_sites, n_sites), dtype=np.uint8)
    L.wldo_all_pairs_dense(_p(buf, ctypes.c_uint8), n_sites, n_seqs, _p(w, ctypes.c_float),
                           _p(d, ctypes.c_float), _p(dp, ctypes.c_float), _p(r2, ctypes.c_float),
                           _p(valid, ctypes.c_uint8))
    return d, dp, r2, valid


_F64_CACHE = {}


def all_pairs_dense_f64(buf, weights):
    """Same sums in double + the epilogue in double: the exact value the f32
    results approximate (diagnostics / accuracy criterion).  The last two
    inputs' results are kept (tests compare several thresholds' rows on one
    alignment against it); treat them as read-only."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    w = np.ascontiguousarray(weights, dtype=np.float32)
    key = (buf.shape, hashlib.sha1(buf.data).hexdigest(), hashlib.sha1(w.data).hexdigest())
    if key not in _F64_CACHE:
        while len(_F64_CACHE) >= 2:
            _F64_CACHE.pop(next(iter(_F64_CACHE)))
        _F64_CACHE[key] = _dense_f64(buf, w)
    return _F64_CACHE[key]


def _dense_f64(buf, w):
    L = lib()
    n_sites, n_seqs = buf.shape
    d = np.zeros((n_sites, n_sites), dtype=np.float64)
    dp = np.zeros_like(d)
    r2 = np.zeros_like(d)
    valid = np.zeros((n_sites, n_sites), dtype=np.uint8)
    L.wldo_all_pairs_dense_f64(_p(buf, ctypes.c_uint8), n_sites, n_seqs, _p(w, ctypes.c_float),
                               _p(d, ctypes.c_double), _p(dp, ctypes.c_double), _p(r2, ctypes.c_double),
                               _p(valid, ctypes.c_uint8))
    return d, dp, r2, valid


def pair_sums_f64(buf, weights):
    """The four masked sums of lib.rs:416-480 for every pair (L x L f64 each:
    T, SA, SB, SAB), with the f32 weights summed in f64 (numpy restatement,
    for conditioning diagnostics)."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    L = buf.shape[0]
    w = np.asarray(weights, dtype=np.float32).astype(np.float64)
    inm = np.zeros(buf.shape, dtype=np.float64)
    mj = np.zeros(buf.shape, dtype=np.float64)
    for s in range(L):
        a, b = major_minor(histogram(buf[s]))
        if a is None or b is None:
            continue
        inm[s] = (buf[s] == a) | (buf[s] == b)
        mj[s] = buf[s] == a
    return (inm * w) @ inm.T, (mj * w) @ inm.T, (inm * w) @ mj.T, (mj * w) @ mj.T


def triu_index(n, i):
    r, c = ctypes.c_size_t(), ctypes.c_size_t()
    lib().wldo_triu_index(n, i, ctypes.byref(r), ctypes.byref(c))
    return r.value, c.value
