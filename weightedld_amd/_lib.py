"""ctypes binding of libweightedld.so (include/weightedld.h).

The shared library is built in-tree by `make` (or __graft_entry__.build()).
There is no Python or CPU fallback for the hot path: if the library is missing
every call raises, and device entry points fail loudly without a gfx950 GPU.
"""
import ctypes
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# WLD_LIB_PATH: an experimental build of the same library (tools/build_variant.sh)
# for the GPU tests of a variant; default the in-tree build
LIB_PATH = os.environ.get("WLD_LIB_PATH") or os.path.join(PKG_DIR, "libweightedld.so")

WLD_OK = 0
STATUS = {
    -1: "WLD_E_ARG",
    -2: "WLD_E_HIP",
    -3: "WLD_E_OOM",
    -4: "WLD_E_NODEV",
    -5: "WLD_E_IO",
    -6: "WLD_E_FORMAT",
    -7: "WLD_E_STATE",
}
KERNEL_AUTO, KERNEL_VALU, KERNEL_MFMA = 0, 1, 2
# wld_set_option ids (include/weightedld.h)
OPTIONS = {"prefilter": 1, "screen": 2, "tile_order": 3, "all_planes": 4, "mfma_layout": 5, "valu_plain": 6,
           "staging_rows": 7, "host_batch_pairs": 8, "ref_sums": 11, "fused_scan": 12, "screen_fp6": 13,
           "test_guard": 14, "fp6_pairs_min_tiles": 15, "i8_pairs": 16}


class WldError(RuntimeError):
    def __init__(self, status, where, message):
        self.status = status
        self.name = STATUS.get(status, str(status))
        super().__init__("%s: %s (%s)" % (where, message, self.name))


class Pairs(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint64),
        ("site_a", ctypes.POINTER(ctypes.c_uint32)),
        ("site_b", ctypes.POINTER(ctypes.c_uint32)),
        ("d", ctypes.POINTER(ctypes.c_float)),
        ("d_prime", ctypes.POINTER(ctypes.c_float)),
        ("r2", ctypes.POINTER(ctypes.c_float)),
    ]


class RunStats(ctypes.Structure):
    _fields_ = [
        ("kernel", ctypes.c_int),
        ("pairs", ctypes.c_uint64),
        ("rows", ctypes.c_uint64),
        ("pair_kernel_ms", ctypes.c_double),
        ("order_ms", ctypes.c_double),
        ("load_ms", ctypes.c_double),
        ("pair_kernel_launches", ctypes.c_uint64),
        ("weight_shift", ctypes.c_int),
        ("mfma_planes", ctypes.c_int),
        ("tiles", ctypes.c_uint64),
        ("candidate_tiles", ctypes.c_uint64),
        ("screen_ms", ctypes.c_double),
        ("screened", ctypes.c_int),
        ("ref_sums", ctypes.c_int),
        ("candidate_blocks", ctypes.c_uint64),
        ("candidate_pairs", ctypes.c_uint64),
        ("screen_fp6", ctypes.c_int),
        ("fp6_sampled", ctypes.c_int),
        ("progress_filled", ctypes.c_uint64),
    ]


PROGRESS_FN = ctypes.CFUNCTYPE(None, ctypes.c_uint64, ctypes.c_void_p)

# name -> (restype, argtypes); every symbol include/weightedld.h declares.
_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_f32p = ctypes.POINTER(ctypes.c_float)
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t
_int = ctypes.c_int
SIGNATURES = {
    "wld_status_string": (ctypes.c_char_p, [_int]),
    "wld_last_error": (ctypes.c_char_p, []),
    "wld_version": (ctypes.c_char_p, []),
    "wld_read_fasta": (_int, [ctypes.c_char_p, ctypes.POINTER(_vp)]),
    "wld_read_vcf": (_int, [ctypes.c_char_p, ctypes.POINTER(_vp)]),
    "wld_siteset_from_buffer": (_int, [_u8p, _sz, _sz, _u64p, ctypes.POINTER(_vp)]),
    "wld_siteset_free": (None, [_vp]),
    "wld_siteset_n_sites": (_sz, [_vp]),
    "wld_siteset_n_seqs": (_sz, [_vp]),
    "wld_siteset_buffer": (_u8p, [_vp]),
    "wld_siteset_site_map": (_u64p, [_vp]),
    "wld_siteset_parent_site_index": (ctypes.c_uint64, [_vp, _sz]),
    "wld_siteset_histogram": (_int, [_vp, _sz, _u64p]),
    "wld_histogram": (_int, [_u8p, _sz, _u64p]),
    "wld_major_minor": (_int, [_u64p, ctypes.POINTER(_int), ctypes.POINTER(_int)]),
    "wld_is_site_of_interest": (_int, [_u8p, _sz, _sz, ctypes.c_float, ctypes.c_float]),
    "wld_siteset_filter_sites_of_interest": (_int, [_vp, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                                    ctypes.POINTER(_vp)]),
    "wld_henikoff_weights": (_int, [_vp, _f32p]),
    "wld_create": (_int, [_int, ctypes.POINTER(_vp)]),
    "wld_create_multi": (_int, [ctypes.POINTER(_int), _int, ctypes.POINTER(_vp)]),
    "wld_n_devices": (_int, [_vp]),
    "wld_destroy": (None, [_vp]),
    "wld_set_kernel": (_int, [_vp, _int]),
    "wld_set_option": (_int, [_vp, _int, ctypes.c_int64]),
    "wld_get_option": (_int, [_vp, _int, ctypes.POINTER(ctypes.c_int64)]),
    "wld_pairs_free": (None, [ctypes.POINTER(Pairs)]),
    "wld_all_weighted_ld_pairs": (_int, [_vp, _u8p, _sz, _sz, _u64p, _f32p, ctypes.c_float, PROGRESS_FN, _vp,
                                         ctypes.POINTER(Pairs)]),
    "wld_single_weighted_ld_pair": (_int, [_vp, _u8p, _u8p, _f32p, _sz, _f32p]),
    "wld_load": (_int, [_vp, _u8p, _sz, _sz, _u64p, _f32p]),
    "wld_load_device": (_int, [_vp, _vp, _sz, _sz, _u64p, _vp]),
    "wld_load_filtered": (_int, [_vp, _u8p, _sz, _sz, _u64p, ctypes.c_float, ctypes.c_float, ctypes.c_float, _int,
                                 ctypes.POINTER(ctypes.c_size_t)]),
    "wld_load_filtered_device": (_int, [_vp, _vp, _sz, _sz, _u64p, ctypes.c_float, ctypes.c_float, ctypes.c_float, _int,
                                        ctypes.POINTER(ctypes.c_size_t)]),
    "wld_weights_copy": (_int, [_vp, _f32p]),
    "wld_site_map_copy": (_int, [_vp, _u64p]),
    "wld_chunk_rows": (ctypes.c_uint32, [_sz]),
    "wld_shard_chunk_rows": (_int, [_sz, _int, _int, _u32p, _u32p]),
    "wld_run": (_int, [_vp, ctypes.c_float, ctypes.c_uint32, ctypes.c_uint32, _u64p]),
    "wld_chunks": (ctypes.c_uint32, [_sz]),
    "wld_shard_chunks": (_int, [_sz, _int, _int, _u32p, _u32p]),
    "wld_pairs_in_chunks": (ctypes.c_uint64, [_sz, ctypes.c_uint32, ctypes.c_uint32]),
    "wld_run_chunks": (_int, [_vp, ctypes.c_float, ctypes.c_uint32, ctypes.c_uint32, _u64p]),
    "wld_run_chunks_async": (_int, [_vp, ctypes.c_float, ctypes.c_uint32, ctypes.c_uint32, _vp]),
    "wld_run_wait": (_int, [_vp, _u64p]),
    "wld_run_after": (_int, [_vp, _vp]),
    "wld_stream": (_vp, [_vp]),
    "wld_set_stream": (_int, [_vp, _vp]),
    "wld_run_host": (_int, [_vp, ctypes.c_float, PROGRESS_FN, _vp, ctypes.POINTER(Pairs)]),
    "wld_rows_device": (_int, [_vp, ctypes.POINTER(Pairs)]),
    "wld_rows_copy": (_int, [_vp, _u32p, _u32p, _f32p, _f32p, _f32p]),
    "wld_rows_copy_device": (_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "wld_dense": (_int, [_vp, _f32p, _f32p, _f32p, _u8p]),
    "wld_last_stats": (_int, [_vp, ctypes.POINTER(RunStats)]),
}

_lib = None


def _preload_torch():
    # torch ships its own libamdhip64.so.7; load it first so this process has
    # exactly one HIP runtime whichever of torch / this library comes first.
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def lib():
    """Loads libweightedld.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise WldError(-2, "load", "%s is missing: run `make` (or __graft_entry__.build())" % LIB_PATH)
    _preload_torch()
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def last_error():
    return lib().wld_last_error().decode(errors="replace")


def check(status, where):
    if status < 0:
        raise WldError(status, where, last_error())
    return status
