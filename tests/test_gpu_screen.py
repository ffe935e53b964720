"""GPU tests of the threshold machinery and the BASELINE configs' parity:

* the r2 prefilter and the one-plane screen (pair_common.hpp r2_bound_skip,
  pair_mfma.hip kModeScreen) never change a row: prefilter/screen on vs off
  bit-identical, on random data, on linkage-block data (many candidate tiles),
  on sites whose minor allele is carried by 1-2 low-weight sequences (the
  near-degenerate denominators where an f32 epilogue is least accurate), at
  thresholds taken from the pairs' own r2 values (rows sitting on the cut),
  and with mixed-sign weights;
* BASELINE config 2 exactly (500 seq x 2000 sites, r2_threshold 0.0: every
  one of the ~2.0M rows against the oracle, in reference order, both kernels);
* weights at the MFMA kernel's dynamic-range boundaries (3 planes down to
  min/max = 2^-4, 4 planes down to 2^-12) at N = 2000 and 5000, the 4-plane
  kernel against the oracle, and a clustered alignment whose Henikoff weights
  span ~2^-11 kept on the integer kernel.
Reference semantics: lib.rs:482-520 (epilogue), :660 (strict r2 > threshold),
:623-683 (row order).
"""
import os
import sys

import numpy as np
import pytest

import _oracle as O
from conftest import REPO
from test_gpu_parity import KERNELS, _ctx, agree, compare_dense, compare_rows, ctxs, dense_check, synth  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def W():
    import weightedld_amd as W
    return W


def _same_rows(a, b):
    for f in ("site_a", "site_b", "d", "d_prime", "r2"):
        x, y = getattr(a, f), getattr(b, f)
        assert len(x) == len(y), (f, len(x), len(y))
        bad = np.nonzero(x.view(np.uint32) != y.view(np.uint32))[0]
        assert len(bad) == 0, (f, len(bad), [(int(a.site_a[i]), int(a.site_b[i]), float(x[i]), float(y[i]),
                                              float(a.r2[i]), float(b.r2[i])) for i in bad[:6]])


def _rows_equal_dense(rows, dense, thr, L):
    """The rows of a run are exactly the dense kernel's pairs with valid and
    r2 > thr (same integer sums, same f32 epilogue), bit for bit, in the
    reference order (chunk in triu_index order, then a, then b)."""
    d, dp, r2, valid = dense
    iu = np.triu_indices(L, 1)
    with np.errstate(invalid="ignore"):
        m = (valid[iu] == 1) & (r2[iu] > np.float32(thr))
    a, b = iu[0][m], iu[1][m]
    n = (L + 255) // 256
    ca, cb = a // 256, b // 256
    rf = n - 1 - ca
    key = (rf * (rf + 1) // 2 + (cb - ca)).astype(np.int64) * L * L + a.astype(np.int64) * L + b
    o = np.argsort(key)
    assert len(rows) == len(o)
    assert np.array_equal(rows.site_a, a[o]) and np.array_equal(rows.site_b, b[o])
    for got, ref in ((rows.d, d), (rows.d_prime, dp), (rows.r2, r2)):
        assert np.array_equal(got.view(np.uint32), ref[a[o], b[o]].view(np.uint32))


def f32_epilogue(T, SA, SB, SAB):
    """lib.rs:482-520 in numpy float32, operation for operation (IEEE,
    no contraction; np.fmax/fmin ignore NaN like Rust's f32::max/min)."""
    f = np.float32
    with np.errstate(all="ignore"):
        PA, PB, o3 = SA, SB, SAB
        Pa, Pb = T - PA, T - PB
        o2, o1 = PA - o3, PB - o3
        o0 = Pa - o1
        PA, PB, Pa, Pb = PA / T, PB / T, Pa / T, Pb / T
        o0, o1, o2, o3 = o0 / T, o1 / T, o2 / T, o3 / T
        d = ((PA * PB - o3) + (Pa * Pb - o0) + (o2 - PA * Pb) + (o1 - Pa * PB)) / f(4)
        neg = d < 0
        den_n = np.fmax(-o0, -o3)
        den_n = np.where(den_n == 0, np.fmin(-o0, -o3), den_n)
        den_p = np.fmin(o1, o2)
        den_p = np.where(den_p == 0, np.fmax(o1, o2), den_p)
        den = np.where(neg, den_n, den_p).astype(f)
        return d, d / den, d * d / (PA * Pa * PB * Pb)


def exact_model_dense(buf, w, shift):
    """What the integer MFMA kernel claims to compute, in numpy: weights as
    fixed point q = rint(w 2^shift), the four masked sums of every pair exact
    (f64 matrix products of integers below 2^53), each rounded once to f32,
    then the reference epilogue in f32.  Returns (d, d', r2, valid)."""
    L, N = buf.shape
    maj = np.full(L, -1)
    mnr = np.full(L, -1)
    for s in range(L):
        a, b = O.major_minor(O.histogram(buf[s]))
        maj[s], mnr[s] = (a, b) if a is not None and b is not None else (-1, -1)
    ok = maj >= 0
    inm = ((buf == maj[:, None]) | (buf == mnr[:, None])) & ok[:, None]
    mj = (buf == maj[:, None]) & ok[:, None]
    q = np.rint(np.ldexp(np.asarray(w, dtype=np.float64), shift))
    i64, m64 = inm.astype(np.float64), mj.astype(np.float64)
    sc = np.ldexp(1.0, -shift)
    T = ((i64 * q) @ i64.T * sc).astype(np.float32)
    SA = ((m64 * q) @ i64.T * sc).astype(np.float32)
    SB = ((i64 * q) @ m64.T * sc).astype(np.float32)
    SAB = ((m64 * q) @ m64.T * sc).astype(np.float32)
    d, dp, r2 = f32_epilogue(T, SA, SB, SAB)
    return d, dp, r2, (ok[:, None] & ok[None, :]).astype(np.uint8)


def check_exact_model(ctx, buf, w, dense=None):
    """GPU dense stats == exact_model_dense, bit for bit (NaN == NaN)."""
    L = buf.shape[0]
    st = ctx.stats()
    assert st["kernel"] == 2  # KERNEL_MFMA
    dense = dense if dense is not None else ctx.dense(L)
    model = exact_model_dense(buf, w, st["weight_shift"])
    iu = np.triu_indices(L, 1)
    assert np.array_equal(dense[3][iu], model[3][iu])
    m = model[3][iu] == 1
    for k, f in enumerate(("d", "d_prime", "r2")):
        g, e = dense[k][iu][m], model[k][iu][m]
        same = (g.view(np.uint32) == e.view(np.uint32)) | (np.isnan(g) & np.isnan(e))
        assert same.all(), (f, int((~same).sum()), g[~same][:4], e[~same][:4])
    return int(m.sum())


def _run(ctx, thr, prefilter, screen):
    ctx.set_option("prefilter", prefilter)
    # 1 -> option 2: the one-plane screen even where auto would not; 3: two planes
    ctx.set_option("screen", {0: 0, 1: 2, 3: 3}[screen])
    ctx.run(thr)
    rows, st = ctx.rows(), ctx.stats()
    ctx.set_option("prefilter", 1)
    ctx.set_option("screen", 1)
    return rows, st


def ld_blocks(L, N, seed, block=40, mut=(0.0, 0.25), p_missing=0.05):
    """Linkage blocks: the sites of a block copy a founder 0/1 pattern with a
    per-site mutation rate, so pairs inside a block have high r2 (many
    candidate tiles for the screen)."""
    rng = np.random.default_rng(seed)
    out = np.empty((L, N), dtype=np.uint8)
    for s0 in range(0, L, block):
        f = rng.random(N) < rng.uniform(0.2, 0.5)
        for s in range(s0, min(L, s0 + block)):
            m = rng.uniform(*mut)
            allele = f ^ (rng.random(N) < m)
            maj, mnr = rng.choice(4, size=2, replace=False)
            col = np.where(allele, mnr, maj)
            out[s] = np.where(rng.random(N) < p_missing, 4, col)
    return out


def rare_carriers(L, N, seed, n_low=8):
    """Sites whose minor allele is carried by 1-3 of n_low low-weight sequences
    (weights 2^-9 .. 2^-5 of the max, inside the MFMA range), plus ordinary
    sites: pairs of rare sites have tiny marginals (Pa ~ 1e-4) — the
    near-degenerate denominators of ADVICE r01."""
    rng = np.random.default_rng(seed)
    w = (0.5 + 0.5 * rng.random(N)).astype(np.float32)
    low = rng.choice(N, size=n_low, replace=False)
    w[low] = (2.0 ** rng.uniform(-9, -5, n_low)).astype(np.float32)
    buf = synth(L, N, seed + 1)
    for s in range(0, L, 2):  # every other site: rare
        maj, mnr = rng.choice(4, size=2, replace=False)
        col = np.full(N, maj, dtype=np.uint8)
        k = rng.integers(1, 4)
        col[rng.choice(low, size=k, replace=False)] = mnr
        if rng.random() < 0.3:  # sometimes one ordinary sequence too
            col[rng.integers(N)] = mnr
        buf[s] = col
    return buf, w


# --------------------------------------------------------------- prefilter/screen
@pytest.mark.parametrize("case", ["random_henikoff", "ld_blocks", "rare_carriers", "mixed_sign"])
def test_prefilter_and_screen_never_change_rows(W, ctxs, case):
    ctx = _ctx(ctxs, "mfma")
    if case == "random_henikoff":
        buf = synth(1500, 1000, 3)
        w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
        thrs = [0.005, 0.01, 0.05, 0.3]
    elif case == "ld_blocks":
        buf = ld_blocks(1200, 800, 4)
        w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
        thrs = [0.05, 0.3, 0.8, 0.95]
    elif case == "rare_carriers":
        buf, w = rare_carriers(900, 2000, 5)
        thrs = [0.05, 0.1, 0.5]
    else:
        buf = synth(700, 600, 6)
        rng = np.random.default_rng(7)
        w = (0.5 + 0.5 * rng.random(600)).astype(np.float32)
        neg = rng.random(600) < 0.1
        w[neg] = -(0.1 + 0.2 * rng.random(int(neg.sum()))).astype(np.float32)
        thrs = [0.01, 0.05, 0.2]
    ctx.load(buf, w)
    assert ctx.stats()["kernel"] == W.KERNEL_MFMA
    # thresholds on the pairs' own r2 values: rows sitting exactly on the cut
    # (one f32 ulp either side of an emitted r2)
    all_rows, _ = _run(ctx, 0.0, 0, 0)
    r2 = all_rows.r2[np.isfinite(all_rows.r2) & (all_rows.r2 > 0.001)]
    if len(r2):
        pick = np.random.default_rng(1).choice(r2, size=min(6, len(r2)), replace=False)
        for v in pick:
            thrs += [float(np.nextafter(v, np.float32(0))), float(v)]
    L = buf.shape[0]
    dense = ctx.dense(L)
    check_exact_model(ctx, buf, w, dense)  # exact sums -> f32 -> reference epilogue, bit for bit
    screened_any = False
    for thr in thrs:
        ref, _ = _run(ctx, thr, 0, 0)       # every pair through the f32 epilogue
        pre, _ = _run(ctx, thr, 1, 0)       # prefilter only
        scr, st = _run(ctx, thr, 1, 1)         # the one-plane i8 screen
        two, st2 = _run(ctx, thr, 1, 3)        # the two-plane i8 screen
        _same_rows(two, ref)
        if ctx.stats()["mfma_planes"] >= 3:
            assert st2["screened"] == 3, st2
            # the top two planes leave a residual 2^8 times smaller
            assert st2["candidate_tiles"] <= st["candidate_tiles"] + 2, (thr, st2, st)
        _same_rows(pre, ref)
        _same_rows(scr, ref)
        _rows_equal_dense(scr, dense, thr, L)
        screened_any |= st["screened"] == 1
        assert st["candidate_tiles"] <= st["tiles"]
    assert screened_any
    # the dense stats against the reference (lib.rs) semantics
    odense, truth = O.all_pairs_dense(buf, w), O.all_pairs_dense_f64(buf, w)[:3]
    if case != "rare_carriers":
        compare_dense(dense, odense, truth)
    else:
        # Outside the reference's own conditioning: a minor cell of ~2^-9
        # weight beside T ~ 1500 lies below one f32 ulp of T, so the
        # epilogue's Pa = (T - PA)/T (lib.rs:482-496) cancels catastrophically
        # in ANY f32 evaluation — the reference's and this kernel's alike
        # (percent-level noise that depends on how the inputs were rounded).
        # There the kernel is pinned by the bit-exact model above (exact sums,
        # the reference epilogue); against the oracle the pairs whose four
        # normalised marginals all exceed 1e-3 must agree strictly, and the
        # rest are counted in the parity report (field "@rare").
        iu = np.triu_indices(L, 1)
        assert np.array_equal(dense[3][iu], odense[3][iu])
        m = odense[3][iu] == 1
        T, SA, SB = O.pair_sums_f64(buf, w)[:3]
        with np.errstate(divide="ignore", invalid="ignore"):
            fmin = np.minimum(np.minimum(SA, T - SA), np.minimum(SB, T - SB)) / T
        well = m & (fmin[iu] > 1e-3)
        compare_dense(dense, odense, truth, mask=well)
        for k, f in enumerate(("d", "d_prime", "r2")):
            agree(dense[k][iu][m & ~well], odense[k][iu][m & ~well], truth[k][iu][m & ~well], field=f + "@rare",
                  escape=True)


def test_screen_auto_policy(W, ctxs):
    # A threshold at which the screen leaves more than half the tiles as
    # candidates (random data, r2 ~ 1/N, thr a few times that) is not screened
    # again, nor is any lower one; higher thresholds still are.  Rows as the
    # oracle's throughout; option 2 screens regardless.
    ctx = _ctx(ctxs, "mfma")
    buf = synth(2000, 2000, 23)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    ctx.load(buf, w)
    assert ctx.get_option("screen") == 1
    ctx.set_option("screen_fp6", 0)  # the i8 tiers' policy (test_gpu_fp6.py: the fp6 screen's handover)
    seen = []
    for thr in (0.002, 0.002, 0.001, 0.05, 0.001, 0.003):
        ctx.run(thr)
        st = ctx.stats()
        seen.append((thr, st["screened"], st["candidate_tiles"], st["tiles"]))
        compare_rows(ctx.rows(), O.all_pairs(buf, w, np.float32(thr)), np.float32(thr), buf=buf, w=w)
    assert seen[0][1] == 1 and seen[0][2] * 2 > seen[0][3], seen
    # 0.002 again: the two-plane screen (3), which leaves more than a fifth
    # (r2 ~ 1/N: most tiles hold a pair above 0.002), so 0.001 goes straight
    # to the full kernel; 0.003 is above the one-plane screen's bad threshold
    assert seen[1][1] == 3 and seen[1][2] * 5 > seen[1][3], seen
    assert [x[1] for x in seen[2:]] == [0, 1, 0, 1], seen
    ctx.set_option("screen", 2)
    rows2 = (ctx.run(0.001), ctx.rows(), ctx.stats()["screened"])
    ctx.set_option("screen", 0)
    rows0 = (ctx.run(0.001), ctx.rows())
    ctx.set_option("screen", 1)
    ctx.set_option("screen_fp6", 1)
    assert rows2[2] == 1 and rows2[0] == rows0[0]
    _same_rows(rows2[1], rows0[1])


def test_two_plane_screen_at_low_threshold(W, ctxs):
    # BASELINE-style random data at thr 0.01 (r2 ~ 1/N, a few pairs per
    # hundred tiles pass): the one-plane screen's residual leaves most tiles
    # undecided, the two-plane screen only a small fraction; rows bit-identical
    # to the unscreened kernel and equal to the oracle's.
    ctx = _ctx(ctxs, "mfma")
    buf = synth(3000, 2000, 31)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    ctx.load(buf, w)
    assert ctx.stats()["mfma_planes"] == 3
    for thr in (0.01, 0.02):
        full, _ = _run(ctx, thr, 1, 0)
        one, st1 = _run(ctx, thr, 1, 1)
        two, st2 = _run(ctx, thr, 1, 3)
        _same_rows(one, full)
        _same_rows(two, full)
        assert st1["screened"] == 1 and st2["screened"] == 3, (st1, st2)
        print("thr %g: candidates one-plane %d, two-plane %d of %d tiles; pair phase %.3f / %.3f ms" % (
            thr, st1["candidate_tiles"], st2["candidate_tiles"], st2["tiles"], st1["pair_kernel_ms"],
            st2["pair_kernel_ms"]))
        assert st2["candidate_tiles"] * 5 < st2["tiles"], st2
        assert st2["candidate_tiles"] < st1["candidate_tiles"], (st1, st2)
        compare_rows(two, O.all_pairs(buf, w, np.float32(thr)), np.float32(thr), buf=buf, w=w)


def test_screen_rejects_random_tiles(W, ctxs):
    # On BASELINE-style random data at 0.05 no pair comes near the cut: the
    # screen must reject (nearly) every tile, so the all-planes launch is tiny.
    ctx = _ctx(ctxs, "mfma")
    buf = synth(3000, 2000, 8)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    ctx.load(buf, w)
    assert ctx.stats()["mfma_planes"] == 3
    n = ctx.run(0.05)
    st = ctx.stats()
    assert st["screened"] == 1 and st["pair_kernel_launches"] == 2
    assert st["candidate_tiles"] <= st["tiles"] // 100, st
    ref = O.all_pairs(buf, w, np.float32(0.05))
    assert n == len(ref["r2"])
    # the screen is skipped where it cannot reject (r2_threshold <= 0); with one
    # digit plane (equal weights) its sums are exact (R = 0) and the candidate
    # launch adds an all-zero plane: same rows as the unscreened kernel
    ctx.run(0.0)
    assert ctx.stats()["screened"] == 0
    ones = np.ones(2000, dtype=np.float32)
    ctx.load(buf, ones)
    for thr in (0.05, 0.004, 0.002):
        n = ctx.run(thr)
        st = ctx.stats()
        assert st["screened"] == 1 and st["mfma_planes"] == 1, st
        rows = ctx.rows()
        un, _ = _run(ctx, thr, 1, 0)
        _same_rows(rows, un)
        compare_rows(rows, O.all_pairs(buf, ones, np.float32(thr)), np.float32(thr), buf=buf, w=ones)


# --------------------------------------------------------------- BASELINE config 2
@pytest.mark.parametrize("kern", KERNELS)
def test_config2_every_row_vs_oracle(W, ctxs, kern):
    """BASELINE configs[1]: synthetic 500 seq x 2000 sites (bench.py's seeded
    generator), Henikoff weights, r2_threshold 0.0 — every row (~2.0M) against
    the oracle, in reference order."""
    sys.path.insert(0, REPO)
    from bench import synth as bench_synth
    ctx = _ctx(ctxs, kern)
    buf = bench_synth(2000, 500)
    ss = W.SiteSet.from_buffer(buf)
    kept = ss.filter_sites_of_interest()
    assert kept.n_sites() == 2000
    w = W.henikoff_weights(kept)
    ctx.load(buf, w)
    n = ctx.run(0.0)
    store = ctx.rows()
    ref = O.all_pairs(buf, w, 0.0)
    assert n == len(store) and n > 1_990_000
    common, only_gpu, only_ref = compare_rows(store, ref, 0.0, buf=buf, w=w)
    # rows on one side only lie within 1e-5 of the cut (compare_rows checks
    # that): pairs at r2 ~ 0, where exact integer sums and the reference's f32
    # sums put r2 on different sides of the strict '> 0.0'
    assert only_gpu + only_ref <= 10 and common == n - only_gpu, (only_gpu, only_ref)
    print("config 2 (%s): %d rows, %d GPU-only, %d reference-only (all within 1e-5 of 0)"
          % (kern, n, only_gpu, only_ref))
    assert ctx.stats()["pairs"] == 2000 * 1999 // 2


# ----------------------------------------------------- wide weight ranges: 4 planes
def clustered(L, N, seed, n_cluster, p_private=0.9, n_private=1):
    """A large identical cluster (tiny Henikoff weights) plus diverse sequences,
    n_private of which carry private symbols at most sites (large weights)."""
    rng = np.random.default_rng(seed)
    maj = rng.integers(0, 4, L)
    mnr = (maj + rng.integers(1, 4, L)) % 4
    third = (mnr + 1) % 4
    third = np.where(third == maj, (third + 1) % 4, third)
    buf = np.repeat(maj[:, None], N, 1).astype(np.uint8)
    div = np.arange(n_cluster, N)
    buf[:, div] = np.where(rng.random((L, len(div))) < 0.3, mnr[:, None], maj[:, None])
    for s in range(L):
        if rng.random() < p_private:
            buf[s, rng.choice(div[:n_private])] = third[s]
    return buf


def test_clustered_alignment_wide_range_on_integer_kernel(W):
    # Henikoff weights spanning ~2^-11 (a 1,900-sequence identical cluster
    # plus 100 diverse): AUTO keeps the integer MFMA kernel with 4 digit planes
    # (31-bit fixed point) instead of the f32 kernel, and matches the oracle.
    import time
    buf = clustered(1500, 2000, 3, 1900, 0.9)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    nz = w[w > 0]
    rng_log2 = float(np.log2(nz.min() / nz.max()))
    assert -12 < rng_log2 < -10, rng_log2
    ctx = W.Context(0, W.KERNEL_AUTO, ref_sums=False)
    ctx.load(buf, w)
    st = ctx.stats()
    assert st["kernel"] == W.KERNEL_MFMA and st["mfma_planes"] == 4, st
    dense_check(ctx, buf, w)
    check_exact_model(ctx, buf, w)
    for thr in (0.0, 0.05):
        t0 = time.perf_counter()
        n = ctx.run(thr)
        dt = time.perf_counter() - t0
        compare_rows(ctx.rows(), O.all_pairs(buf, w, np.float32(thr)), np.float32(thr), buf=buf, w=w)
        print("clustered 1500 sites x 2000 seqs (weights 2^%.2f): thr %g, %d rows, pair phase %.3f ms "
              "(screened %d), run %.1f ms" % (rng_log2, thr, n, ctx.stats()["pair_kernel_ms"],
                                               ctx.stats()["screened"], dt * 1e3))
    # the f32 kernel on the same input, for the record
    v = W.Context(0, W.KERNEL_VALU, ref_sums=False)
    v.load(buf, w)
    v.run(0.0)
    print("  f32 kernel: pair phase %.3f ms" % v.stats()["pair_kernel_ms"])


@pytest.mark.parametrize("spread", [2.0 ** -6, 2.0 ** -11])
def test_four_plane_kernel_vs_oracle(W, ctxs, spread):
    # weights in [spread, 1]: 4 digit planes; dense stats and rows (both
    # through the screen at 0.02 and unscreened) against the oracle
    ctx = _ctx(ctxs, "mfma")
    rng = np.random.default_rng(int(-np.log2(spread)))
    buf = synth(700, 900, 12)
    w = np.exp(rng.uniform(np.log(spread), 0.0, 900)).astype(np.float32)
    w[0] = 1.0
    w[1] = np.float32(spread)
    ctx.load(buf, w)
    assert ctx.stats()["mfma_planes"] == 4
    dense_check(ctx, buf, w)
    check_exact_model(ctx, buf, w)
    for thr in (0.0, 0.02):
        ctx.run(thr)
        compare_rows(ctx.rows(), O.all_pairs(buf, w, np.float32(thr)), np.float32(thr), buf=buf, w=w)


# ------------------------------------------------------- MFMA dynamic-range boundary
@pytest.mark.parametrize("N", [2000, 5000])
@pytest.mark.parametrize("spread,planes", [(2.0 ** -4, 3), (2.0 ** -10, 4), (2.0 ** -12, 4)])
def test_weights_at_mfma_range_boundary(W, N, spread, planes):
    # min/max just above each AUTO boundary (2^-4: 3 planes; 2^-12: 4 planes;
    # the old 2^-10 cut): the smallest weights are quantised most coarsely
    # (0.5 / q_min <= 2^-19 relative), and half the weights identical and small
    # make their rounding errors add coherently.  Just below 2^-12: f32 kernel.
    rng = np.random.default_rng(N)
    buf = synth(300, N, N + 1)
    w = (0.5 + 0.5 * rng.random(N)).astype(np.float32)
    w[0] = 1.0
    small = rng.random(N) < 0.5
    small[0] = False
    w[small] = np.float32(spread * (1 + 2.0 ** -12))
    ctx = W.Context(0, W.KERNEL_AUTO, ref_sums=False)
    ctx.load(buf, w)
    assert ctx.stats()["kernel"] == W.KERNEL_MFMA and ctx.stats()["mfma_planes"] == planes
    dense_check(ctx, buf, w)
    check_exact_model(ctx, buf, w)
    ctx.run(0.01)
    compare_rows(ctx.rows(), O.all_pairs(buf, w, 0.01), 0.01, buf=buf, w=w)
    if spread == 2.0 ** -12:
        w[small] = np.float32(spread * (1 - 2.0 ** -12))
        ctx.load(buf, w)
        assert ctx.stats()["kernel"] == W.KERNEL_VALU


@pytest.mark.parametrize("opts", [{}, {"screen_fp6": 0}, {"screen_fp6": 2}, {"ref_sums": 0}],
                         ids=["auto", "i8", "fp6", "exact_sums"])
def test_guard_refuses_corrupt_candidate_entry(W, opts):
    """a candidate entry outside the screen's buckets is refused by
    the candidate launch's guard (cand_entry_checked) and the run fails with
    WLD_E_STATE instead of reading through it (WLD_OPT_TEST_GUARD corrupts the
    last bucket's count between the screen and the candidate launch); the
    next run is clean and its rows equal the oracle's."""
    L, N, thr = 900, 300, 0.2
    buf = synth(L, N, 11)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    ref = O.all_pairs(buf, w, np.float32(thr))
    c = W.Context(0, W.KERNEL_MFMA)
    for k, v in opts.items():
        c.set_option(k, v)
    c.load(buf, w)
    c.run(thr)
    compare_rows(c.rows(), ref, thr, buf=buf, w=w)
    assert c.stats()["screened"] == 1
    c.set_option("test_guard", 1)
    with pytest.raises(W.WldError) as e:
        c.run(thr)
    assert e.value.name == "WLD_E_STATE", e.value
    assert "out-of-range" in str(e.value), e.value
    c.set_option("test_guard", 0)
    c.run(thr)
    compare_rows(c.rows(), ref, thr, buf=buf, w=w)
    c.close()
