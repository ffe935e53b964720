"""The fp6 screen (pair_mfma.hip pair_fp6_screen_kernel, WLD_OPT_SCREEN_FP6):
the one-plane screen's sums on block-scaled fp6 x fp4 MFMA.  A screen only
decides which tiles the candidate launch computes, so rows must be
bit-identical to the i8 screen's, to the unscreened kernel's and (the default,
lib.rs's summation order) to the oracle's, on every data kind — including
linkage blocks and rare alleles, where many tiles are candidates and the
screen's residual bound is what keeps a passing pair from being skipped.
Reference semantics: lib.rs:482-520 (epilogue), :660 (strict r2 > thr),
:623-683 (row order).
"""
import numpy as np
import pytest

import _oracle as O
from conftest import REPO  # noqa: F401
from test_gpu_parity import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def W():
    import weightedld_amd as W
    return W


def _bits_equal(store, ref):
    assert len(store) == len(ref["site_a"]), (len(store), len(ref["site_a"]))
    assert np.array_equal(store.site_a.astype(np.uint64), ref["site_a"].astype(np.uint64))
    assert np.array_equal(store.site_b.astype(np.uint64), ref["site_b"].astype(np.uint64))
    for f in ("d", "d_prime", "r2"):
        x, y = getattr(store, f), np.asarray(ref[f], dtype=np.float32)
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32)), f


def _store_dict(s):
    return {f: getattr(s, f) for f in ("site_a", "site_b", "d", "d_prime", "r2")}


def _data(kind, L, N, seed):
    import bench
    rng = np.random.default_rng(seed)
    if kind == "random":
        buf = synth(L, N, seed)
    elif kind == "ldblocks":
        buf = bench.ld_blocks(L, N, seed=seed)
    elif kind == "rare":
        buf = synth(L, N, seed)
        for s in range(0, L, 3):  # minor allele on 1-3 sequences
            buf[s] = np.where(buf[s] == 4, 4, 0)
            buf[s, rng.choice(N, size=int(rng.integers(1, 4)), replace=False)] = 1
    else:
        raise ValueError(kind)
    return buf


@pytest.mark.parametrize("kind", ["random", "ldblocks", "rare"])
@pytest.mark.parametrize("weights", ["henikoff", "wide", "unit"])
def test_fp6_screen_rows_bit_identical(W, kind, weights):
    L, N = 1500, 700
    buf = _data(kind, L, N, 17)
    if weights == "henikoff":
        w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    elif weights == "wide":  # 16x range: the fp6 rounding's relative error is largest
        w = (np.random.default_rng(5).random(N) * 15 + 1).astype(np.float32)
    else:
        w = np.ones(N, dtype=np.float32)
    ctxs = {}
    # fp6 on the single-tile kernel (a list under fp6_pairs_min_tiles) and on
    # the tile-pair kernel (fp6_pairs_min_tiles 0, the default), and the i8 screen
    for name, fp6, pairs_min in (("fp6", 2, 1 << 30), ("fp6pairs", 2, 0), ("i8", 0, None)):
        c = W.Context(0)
        c.set_option("screen_fp6", fp6)
        if pairs_min is not None:
            c.set_option("fp6_pairs_min_tiles", pairs_min)
        c.load(buf, w)
        ctxs[name] = c
    for thr in (0.05, 0.2, 0.01, 0.5):
        ref = O.all_pairs(buf, w, np.float32(thr))
        out = {}
        for name, c in ctxs.items():
            n = c.run(thr)
            st = c.stats()
            out[name] = (c.rows(), st)
            assert n == len(ref["site_a"])
            _bits_equal(out[name][0], ref)
        for k in ("fp6", "fp6pairs"):
            st6 = out[k][1]
            if st6["screened"] == 1:
                assert st6["screen_fp6"] == 1, st6
        assert out["i8"][1]["screen_fp6"] == 0
    for c in ctxs.values():
        c.close()


def test_fp6_exact_mode_rows(W):
    """Exact sums (WLD_OPT_REF_SUMS 0): the candidate launch's integer kernel
    behind the fp6 screen gives the same rows as without any screen."""
    L, N = 1300, 900
    buf = _data("ldblocks", L, N, 23)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    a, b = W.Context(0, ref_sums=False), W.Context(0, ref_sums=False)
    a.set_option("screen_fp6", 2)
    b.set_option("screen", 0)
    a.load(buf, w)
    b.load(buf, w)
    for thr in (0.05, 0.3):
        assert a.run(thr) == b.run(thr)
        assert a.stats()["screen_fp6"] == 1
        _bits_equal(a.rows(), _store_dict(b.rows()))


def test_fp6_handover_to_i8(W):
    """Auto policy: at a threshold where the fp6 screen reaches a sixteenth of
    the tiles as candidates it gives the pass up and the pass re-runs on the i8
    screen (screen_fp6 2), or (one round of tiles) completes; that threshold
    and any lower one screen on i8 from then on; higher thresholds stay on
    fp6.  Rows equal the oracle's throughout."""
    import bench
    buf = bench.synth(2048, 2000)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    c = W.Context(0)
    c.load(buf, w)
    seen = []
    for thr in (0.002, 0.002, 0.001, 0.05):
        c.run(thr)
        st = c.stats()
        seen.append((thr, st["screened"], st["screen_fp6"], st["candidate_tiles"], st["tiles"]))
        _bits_equal(c.rows(), O.all_pairs(buf, w, np.float32(thr)))
    # (a grid of one round of workgroups cannot give up: every workgroup has
    # read the count before the first candidate lands; the pass then
    # completes and hands over by its count)
    assert seen[0][2] == 2 or (seen[0][2] == 1 and seen[0][3] * 16 > seen[0][4]), seen
    assert seen[1][2] == 0 and seen[2][2] == 0 and seen[3][1:3] == (1, 1), seen
    c.close()


def test_fp6_sample_run_on_ld_blocks(W):
    """Linkage blocks, auto (WLD_OPT_SCREEN_FP6 1): the fp6 screen's sample
    run (about 1/64 of the tiles, counting only) finds nearly every sampled
    tile a candidate, so the first pass at that threshold already screens on
    i8 (no pass is given up), and so does a lower threshold with no new
    sample; on the bench's random data the sample keeps fp6, and a higher
    threshold needs no new sample.  Rows equal the oracle's throughout."""
    import bench
    L, N, thr = 4096, 2000, 0.05
    buf = bench.ld_blocks(L, N, seed=7)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    c = W.Context(0)
    c.load(buf, w)
    for t, sampled in ((thr, 1), (0.03, 0), (thr, 0)):
        c.run(t)
        st = c.stats()
        assert st["fp6_sampled"] == sampled and st["screen_fp6"] == 0 and st["screened"] in (1, 3, 4), (t, st)
        _bits_equal(c.rows(), O.all_pairs(buf, w, np.float32(t)))
    buf = bench.synth(L, N)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    c.load(buf, w)
    for t, sampled in ((0.05, 1), (0.1, 0), (0.05, 0)):
        c.run(t)
        st = c.stats()
        assert st["fp6_sampled"] == sampled and st["screen_fp6"] == 1, (t, st)
        _bits_equal(c.rows(), O.all_pairs(buf, w, np.float32(t)))
    c.close()


def test_fp6_abandoned_pass_on_ld_blocks(W):
    """Linkage blocks: nearly every tile holds a pair the fp6 bound (1.4%
    residual on these weights) cannot reject.  Auto without the sample run
    (WLD_OPT_SCREEN_FP6 3, the safety net behind it): the first pass gives up
    after a sixteenth of the tiles and re-runs on i8 inside the same call;
    rows equal the oracle's.  With per-chunk progress, or a caller's count
    word (the N>1 step's collective reads it), the pass is never given up:
    the fp6 screen completes, its candidates are computed, and the next pass
    hands over by the candidate count."""
    import bench
    import torch
    L, N, thr = 4096, 2000, 0.05
    buf = bench.ld_blocks(L, N, seed=7)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    ref = O.all_pairs(buf, w, np.float32(thr))
    assert len(ref["site_a"]) > 1000
    c = W.Context(0)
    c.set_option("screen_fp6", 3)
    c.load(buf, w)
    c.run(thr)
    st = c.stats()
    assert st["screen_fp6"] == 2 and st["screened"] in (1, 3, 4), st
    _bits_equal(c.rows(), ref)
    c.run(thr)
    assert c.stats()["screen_fp6"] == 0
    _bits_equal(c.rows(), ref)
    # progress: no give-up
    c.load(buf, w)
    calls = []
    store = c.run_host(thr, calls.append)
    st = c.stats()
    assert st["screen_fp6"] == 1 and st["candidate_tiles"] * 16 > st["tiles"], st
    assert calls and calls[0] == 0
    _bits_equal(store, ref)
    c.run(thr)
    assert c.stats()["screen_fp6"] == 0
    # a caller's count word: no give-up either
    c.load(buf, w)
    cnt = torch.full((1,), -1, dtype=torch.int64, device="cuda:0")
    c.run_chunks_async(thr, 0, 0, cnt.data_ptr())
    n = c.run_wait()
    torch.cuda.synchronize()
    assert n == int(cnt.item()) == len(ref["site_a"])
    assert c.stats()["screen_fp6"] == 1
    _bits_equal(c.rows(), ref)
    c.close()


def test_fp6_default_on_bench_data_and_ineligible_weights(W):
    """Auto: the bench's Henikoff weights (nearly equal) take the fp6 screen;
    mixed-sign weights never do (its bound assumes nonnegative cells)."""
    import bench
    buf = bench.synth(2048, 2000)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    c = W.Context(0)
    c.load(buf, w)
    c.run(0.05)
    st = c.stats()
    # (at 2,048 sites the weights spread more than at C4's 20,000: the fp6
    # rounding leaves ~1.4% of the sums, and a few tiles stay candidates)
    assert st["screened"] == 1 and st["screen_fp6"] == 1 and st["candidate_tiles"] * 10 <= st["tiles"], st
    _bits_equal(c.rows(), O.all_pairs(buf, w, np.float32(0.05)))
    wm = w.copy()
    wm[::7] *= -1
    c.load(buf, wm)
    c.run(0.05)
    assert c.stats()["screen_fp6"] == 0
    _bits_equal(c.rows(), O.all_pairs(buf, wm, np.float32(0.05)))
    c.close()


@pytest.mark.parametrize("pairs", [False, True])
@pytest.mark.parametrize("N", [64, 100, 128, 190, 1000, 2049])
def test_fp6_sequence_counts(W, N, pairs):
    """NP not a multiple of 128 (a zero-padded last fp6 block), tiny N; on the
    single-tile (forced) and tile-pair kernels (L 700: 11 tile rows, so the
    pair list holds single entries beside pairs)."""
    L = 700
    buf = synth(L, N, 31 + N)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    c = W.Context(0)
    c.set_option("screen_fp6", 2)
    c.set_option("fp6_pairs_min_tiles", 0 if pairs else 1 << 30)
    c.load(buf, w)
    for thr in (0.02, 0.1):
        c.run(thr)
        _bits_equal(c.rows(), O.all_pairs(buf, w, np.float32(thr)))
    c.close()


@pytest.mark.parametrize("cfg", ["c4", "c5"])
def test_fp6_forced_full_size_rows(W, cfg):
    """The headline kernel where it can fail: the fp6 screen forced
    (WLD_OPT_SCREEN_FP6 2: the pass always completes, never hands over to i8)
    on BASELINE configs 4 and 5 at full size (the bench's own seeded inputs,
    Henikoff weights: 313 / 782 tile rows, every tile of the XCD-ordered
    list), at thresholds where rows pass: >= 1,000 oracle rows at C4, >= 10^4
    at C5.  The pass must run on fp6 (stats screen_fp6 1), and its rows,
    their order and every bit of d, d', r2 equal the oracle's (lib.rs:482-520,
    :660, :623-683).  One oracle run at the lowest threshold; the others are
    its strict-'>' subsets."""
    import bench
    N, L, thr, _ = bench.CONFIGS[cfg]
    buf = bench.synth(L, N)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    thrs = (0.02, 0.015, 0.01) if cfg == "c4" else (0.01, 0.005, 0.004)
    lo = np.float32(min(thrs))
    ref = O.all_pairs(buf, w, lo)
    assert ref["pairs"] == L * (L - 1) // 2
    c = W.Context(0)
    c.set_option("screen_fp6", 2)
    c.load(buf, w)
    counts = []
    for t in thrs:
        t32 = np.float32(t)
        sub = {f: v[ref["r2"] > t32] for f, v in ref.items() if f != "pairs"}
        n = c.run(t)
        st = c.stats()
        assert st["screened"] == 1 and st["screen_fp6"] == 1, st
        assert n == len(sub["r2"])
        _bits_equal(c.rows(), sub)
        counts.append((t, n, st["candidate_tiles"], st["tiles"]))
    print("fp6 forced full size %s: (thr, rows, candidate tiles, tiles) %s" % (cfg, counts))
    assert max(n for _, n, _, _ in counts) >= (1000 if cfg == "c4" else 10000), counts
    c.close()


def _planted(cfg):
    import bench
    N, L, thr, _ = bench.CONFIGS[cfg]
    buf, planted = bench.planted_ld(L, N)
    import weightedld_amd as W
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    return buf, w, np.float32(thr), planted


@pytest.fixture(scope="module")
def planted_c4():
    buf, w, thr, planted = _planted("c4")
    return buf, w, thr, planted, O.all_pairs(buf, w, thr)


@pytest.mark.parametrize("mode", ["forced", "auto"])
def test_fp6_planted_full_size_c4(W, planted_c4, mode):
    """the headline screen where it rejects nearly every tile
    yet must keep the few that hold rows.  BASELINE config 4 at full size and
    its threshold 0.05, the bench's seeded background with planted linkage
    (bench.planted_ld: ~750 passing pairs over ~380 tiles on every XCD queue,
    both halves of tile-pair entries, single entries, diagonal tiles and the
    padded last tile row and column; r2 from 1 down to just above 0.05, and
    planted pairs just below it).  fp6 forced (WLD_OPT_SCREEN_FP6 2) and auto
    (the sample run decides): the pass runs on fp6, candidates are <= 2% of
    the tiles, and the rows, their order and every bit of d, d', r2 equal the
    oracle's (lib.rs:647-669, :660), twice on one context."""
    buf, w, thr, planted, ref = planted_c4
    L = buf.shape[0]
    rt = set(zip((ref["site_a"] // 64).tolist(), (ref["site_b"] // 64).tolist()))
    assert len(ref["r2"]) >= 500 and len(rt) >= 300, (len(ref["r2"]), len(rt))
    T = (L + 63) // 64
    assert any(a == b for a, b in rt) and any(b == T - 1 for _, b in rt) and (T - 1, T - 1) in rt
    c = W.Context(0)
    if mode == "forced":
        c.set_option("screen_fp6", 2)
    c.load(buf, w)
    seen = []
    for _ in range(2):
        n = c.run(float(thr))
        st = c.stats()
        seen.append((n, st["candidate_tiles"], st["candidate_blocks"], st["tiles"], st["fp6_sampled"]))
        assert st["screened"] == 1 and st["screen_fp6"] == 1, st
        assert st["candidate_tiles"] * 50 <= st["tiles"], st
        assert st["candidate_tiles"] >= len(rt), (st, len(rt))
        assert n == len(ref["r2"])
        _bits_equal(c.rows(), ref)
    print("planted C4 %s: rows %d over %d tiles; (rows, candidate tiles, candidate sub-blocks, tiles, sampled) %s"
          % (mode, len(ref["r2"]), len(rt), seen))
    c.close()


def test_fp6_planted_full_size_c5(W):
    """The same at BASELINE config 5's size (5000 x 50000, thr 0.05), where
    the full oracle does not fit a test's time: the forced-fp6 and auto rows
    equal, bit for bit, those of the unscreened run (every tile through the
    kernel in lib.rs's summation order, WLD_OPT_SCREEN 0 — the path the
    oracle pins at every smaller size), and every planted pair's d, d', r2
    equal the oracle's single_weighted_ld_pair (lib.rs:390-521); every
    planted pair with r2 > thr is a row."""
    buf, w, thr, planted = _planted("c5")
    ref_c = W.Context(0)
    ref_c.set_option("screen", 0)
    ref_c.load(buf, w)
    n_ref = ref_c.run(float(thr))
    ref = _store_dict(ref_c.rows())
    ref_c.close()
    rows = {(int(a), int(b)): i for i, (a, b) in enumerate(zip(ref["site_a"], ref["site_b"]))}
    hits = 0
    for a, b, _ in planted:
        d, dp, r2 = O.single_pair(buf[a], buf[b], w)
        if np.float32(r2) > thr:
            i = rows[(a, b)]
            got = np.array([ref["d"][i], ref["d_prime"][i], ref["r2"][i]], dtype=np.float32)
            assert np.array_equal(got.view(np.uint32), np.array([d, dp, r2], dtype=np.float32).view(np.uint32))
            hits += 1
    rt = set(zip((ref["site_a"] // 64).tolist(), (ref["site_b"] // 64).tolist()))
    assert hits >= 500 and len(rt) >= 300, (hits, len(rt))
    for mode in ("forced", "auto"):
        c = W.Context(0)
        if mode == "forced":
            c.set_option("screen_fp6", 2)
        c.load(buf, w)
        n = c.run(float(thr))
        st = c.stats()
        assert st["screened"] == 1 and st["screen_fp6"] == 1, st
        assert st["candidate_tiles"] * 50 <= st["tiles"], st
        assert n == n_ref
        _bits_equal(c.rows(), ref)
        print("planted C5 %s: rows %d (planted %d) over %d tiles; candidate tiles %d of %d"
              % (mode, n, hits, len(rt), st["candidate_tiles"], st["tiles"]))
        c.close()
