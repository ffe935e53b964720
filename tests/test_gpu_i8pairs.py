"""The i8 one-plane screen on tile pairs with wide waves (pair_mfma.hip
pair_i8_screen2w_kernel, WLD_OPT_I8_PAIRS 1, round 6): the screen the
linkage-structured data runs on where the fp6 rounding is too coarse.  A
screen only decides which tiles the candidate launch computes, so with the
i8 screen forced (WLD_OPT_SCREEN_FP6 0) the rows must be bit-identical to the
per-tile i8 kernel's (WLD_OPT_I8_PAIRS 0) and to the oracle's (lib.rs's
summation order), on random, linkage-block and rare-allele data, Henikoff,
wide-range and unit weights, sequence counts that leave a zero-padded last
64-sequence block, and at full size (BASELINE config 4 with planted linkage,
and C4-size linkage blocks with the auto policy).  Reference semantics:
lib.rs:482-520 (epilogue), :660 (strict r2 > thr), :623-683 (row order).
"""
import numpy as np
import pytest

import _oracle as O
from conftest import REPO  # noqa: F401
from test_gpu_fp6 import _bits_equal, _data, _store_dict

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def W():
    import weightedld_amd as W
    return W


def _weights(W, buf, kind):
    N = buf.shape[1]
    if kind == "unit":
        return np.ones(N, dtype=np.float32)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    if kind == "wide":
        w = w.copy()
        w[::5] *= np.float32(1.0 / 16)
    return w


@pytest.mark.parametrize("kind", ["random", "ldblocks", "rare"])
@pytest.mark.parametrize("weights", ["henikoff", "wide", "unit"])
def test_i8_pair_screen_rows_bit_identical(W, kind, weights):
    L, N = 1500, 700
    buf = _data(kind, L, N, 91)
    w = _weights(W, buf, weights)
    a, b = W.Context(0), W.Context(0)
    for c in (a, b):
        c.set_option("screen_fp6", 0)
        c.set_option("screen", 2)  # the one-plane screen at every threshold
    b.set_option("i8_pairs", 0)
    a.load(buf, w)
    b.load(buf, w)
    for thr in (0.02, 0.05, 0.2, 0.6):
        na, nb = a.run(thr), b.run(thr)
        sa, sb = a.stats(), b.stats()
        assert sa["screened"] == 1 and sa["screen_fp6"] == 0, sa
        assert na == nb
        _bits_equal(a.rows(), _store_dict(b.rows()))
        _bits_equal(a.rows(), O.all_pairs(buf, w, np.float32(thr)))
        # the same sums, the bound on exact marginals with R2 = 2R rounded up
        # to the integer grid (the per-tile kernel: R rounded up in f32): about
        # the same candidate tiles
        assert abs(sa["candidate_tiles"] - sb["candidate_tiles"]) <= max(2, sb["candidate_tiles"] // 50), (sa, sb)
    a.close()
    b.close()


@pytest.mark.parametrize("N", [64, 100, 190, 1000, 2049])
def test_i8_pair_screen_sequence_counts(W, N):
    """NP a multiple of 64 (a zero-padded last block), tiny N; L 700: 11
    tile rows, so the pair list holds single entries beside pairs."""
    L = 700
    buf = _data("ldblocks", L, N, 5 + N)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    c = W.Context(0)
    c.set_option("screen_fp6", 0)
    c.set_option("screen", 2)
    c.load(buf, w)
    for thr in (0.05, 0.3):
        c.run(thr)
        assert c.stats()["screened"] == 1
        _bits_equal(c.rows(), O.all_pairs(buf, w, np.float32(thr)))
    c.close()


def test_i8_pair_screen_planted_full_size(W):
    """BASELINE config 4 at full size and threshold with planted linkage
    (bench.planted_ld), the i8 screen forced: candidate tiles <= 2% of the
    tiles and every tile holding a row among them, rows equal to the
    oracle's bit for bit."""
    import bench
    N, L, thr, _ = bench.CONFIGS["c4"]
    buf, _ = bench.planted_ld(L, N)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    ref = O.all_pairs(buf, w, np.float32(thr))
    rt = set(zip((ref["site_a"] // 64).tolist(), (ref["site_b"] // 64).tolist()))
    c = W.Context(0)
    c.set_option("screen_fp6", 0)
    c.load(buf, w)
    n = c.run(thr)
    st = c.stats()
    assert st["screened"] == 1 and st["screen_fp6"] == 0, st
    assert len(rt) <= st["candidate_tiles"] <= st["tiles"] // 50, (st, len(rt))
    assert n == len(ref["r2"]) >= 500
    _bits_equal(c.rows(), ref)
    print("planted C4 on the i8 pair screen: rows %d over %d tiles, candidate tiles %d of %d"
          % (n, len(rt), st["candidate_tiles"], st["tiles"]))
    c.close()


def test_i8_pair_screen_ld_blocks_c4_auto(W):
    """C4-size linkage blocks (bench --data ldblocks), the default policy:
    the fp6 sample hands the threshold to the i8 screen, which runs on tile
    pairs; rows equal the oracle's bit for bit (~700,000 rows)."""
    import bench
    N, L, thr, _ = bench.CONFIGS["c4"]
    buf = bench.ld_blocks(L, N)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    ref = O.all_pairs(buf, w, np.float32(thr))
    c = W.Context(0)
    c.load(buf, w)
    for _ in range(2):
        n = c.run(thr)
        st = c.stats()
        assert st["screened"] == 1 and st["screen_fp6"] == 0, st
        assert n == len(ref["r2"]) > 100_000
        _bits_equal(c.rows(), ref)
    print("C4 linkage blocks: rows %d, candidate tiles %d of %d" % (n, st["candidate_tiles"], st["tiles"]))
    c.close()
