"""GPU tests of the reference summation order (WLD_OPT_REF_SUMS) and of how
far the exact-sum path's rows lie from lib.rs's on ill-conditioned inputs.

lib.rs sums each pair's four masked weights in f32 in its own order: 8 lane
sums over sequences k = j mod 8 (lib.rs:416-445), their horizontal sum
(:447-452), then the scalar tail (:461-480).  The exact-sum path
(WLD_OPT_REF_SUMS 0) sums exactly (integer MFMA) and rounds once, which is
more accurate but differs from lib.rs by lib.rs's own rounding — far beyond
1e-5 where a minor allele is carried by a few low-weight sequences.  With
WLD_OPT_REF_SUMS 1 (the default) the f32 kernel
adds the same terms in the same order (sequences permuted into lane classes,
the ordered horizontal sum packed_simd's x86 f32x8::sum() computes), so
d, d' and r2 must be BIT-identical to the oracle's (oracle/wld_oracle.c, the
C restatement of lib.rs with the same order) — on every pair, every input,
with or without the i8 screen in front.

The report tests print, per input, the exact-sum path's (WLD_OPT_REF_SUMS 0)
row-set and %.3f TSV-line differences against the oracle, and the
reference-order path's (the default) against the oracle under both
horizontal-sum orders (ordered, packed_simd's
implementation; tree, its documentation): tests/conftest.py REF_REPORT.
"""
import sys

import numpy as np
import pytest

import _oracle as O
from conftest import REF_REPORT, REPO
from test_gpu_parity import synth
from test_gpu_screen import ld_blocks, rare_carriers

pytestmark = pytest.mark.gpu
sys.path.insert(0, REPO)
import bench  # noqa: E402  (the seeded generators of the bench workloads)


@pytest.fixture(scope="module")
def W():
    import weightedld_amd as W
    return W


@pytest.fixture(scope="module")
def ref_ctx(W):
    c = W.Context(0, W.KERNEL_AUTO)
    c.set_option("ref_sums", 1)
    return c


def _bits_equal(g, r):
    g = np.ascontiguousarray(g, dtype=np.float32)
    r = np.ascontiguousarray(r, dtype=np.float32)
    return (g.view(np.uint32) == r.view(np.uint32)) | (np.isnan(g) & np.isnan(r))


def assert_dense_bit_exact(ctx, buf, w):
    L = buf.shape[0]
    d, dp, r2, valid = ctx.dense(L)
    od, odp, or2, ovalid = O.all_pairs_dense(buf, w)
    iu = np.triu_indices(L, 1)
    assert np.array_equal(valid[iu], ovalid[iu])
    m = ovalid[iu] == 1
    for f, g, r in (("d", d, od), ("d_prime", dp, odp), ("r2", r2, or2)):
        same = _bits_equal(g[iu][m], r[iu][m])
        assert same.all(), (f, int((~same).sum()), g[iu][m][~same][:5], r[iu][m][~same][:5])
    assert ctx.stats()["ref_sums"] == 1
    return int(m.sum())


def _keys(a, b):
    return np.asarray(a, dtype=np.uint64) << np.uint64(32) | np.asarray(b, dtype=np.uint64)


def assert_rows_bit_exact(store, ref):
    assert len(store) == len(ref["site_a"]), (len(store), len(ref["site_a"]))
    assert np.array_equal(store.site_a.astype(np.uint64), ref["site_a"])
    assert np.array_equal(store.site_b.astype(np.uint64), ref["site_b"])
    for f in ("d", "d_prime", "r2"):
        same = _bits_equal(getattr(store, f), ref[f])
        assert same.all(), (f, int((~same).sum()))


def row_diff(store, ref, thr, tol=1e-5):
    """Row-set and value differences of GPU rows against oracle rows:
    rows on one side only (and how many of them lie outside the +-tol band
    around thr, i.e. are not explained by a strict '>' on sums rounded
    differently), values beyond tol among common rows, %.3f TSV lines that
    differ (main.rs:101-108; one-sided rows count as differing lines)."""
    kg = _keys(store.site_a, store.site_b)
    kr = _keys(ref["site_a"], ref["site_b"])
    _, ig, ir = np.intersect1d(kg, kr, assume_unique=True, return_indices=True)
    only_g = np.setdiff1d(np.arange(len(kg)), ig)
    only_r = np.setdiff1d(np.arange(len(kr)), ir)
    out_band = int((np.abs(store.r2[only_g].astype(np.float64) - thr) > tol).sum() +
                   (np.abs(ref["r2"][only_r].astype(np.float64) - thr) > tol).sum())
    res = {"rows_gpu": len(kg), "rows_ref": len(kr), "only_gpu": len(only_g), "only_ref": len(only_r),
           "one_sided_outside_band": out_band}
    tsv_diff = 0
    lines_g, lines_r = None, None
    for f in ("d", "d_prime", "r2"):
        g = getattr(store, f)[ig].astype(np.float64)
        r = ref[f][ir].astype(np.float64)
        with np.errstate(invalid="ignore"):
            dif = np.abs(g - r)
            bad = ~((dif <= tol * np.maximum(1.0, np.abs(r))) | (np.isnan(g) & np.isnan(r)))
        res["beyond_tol_" + f] = int(bad.sum())
        res["max_diff_" + f] = float(np.nanmax(dif)) if len(dif) else 0.0
        fg = np.char.mod("%.3f", getattr(store, f)[ig].astype(np.float64))
        fr = np.char.mod("%.3f", ref[f][ir].astype(np.float64))
        lines_g = fg if lines_g is None else np.char.add(np.char.add(lines_g, "\t"), fg)
        lines_r = fr if lines_r is None else np.char.add(np.char.add(lines_r, "\t"), fr)
    if len(ig):
        tsv_diff = int((lines_g != lines_r).sum())
    res["tsv_lines_differing"] = tsv_diff + len(only_g) + len(only_r)
    return res


def _fmt(name, mode, res):
    return ("%-34s %-22s rows %d/%d (gpu/ref), one-sided %d+%d (%d outside +-1e-5 of thr), beyond 1e-5: d %d d' %d "
            "r2 %d (max |diff| d %.2g d' %.2g r2 %.2g), TSV lines differing %d" % (
                name, mode, res["rows_gpu"], res["rows_ref"], res["only_gpu"], res["only_ref"],
                res["one_sided_outside_band"], res["beyond_tol_d"], res["beyond_tol_d_prime"], res["beyond_tol_r2"],
                res["max_diff_d"], res["max_diff_d_prime"], res["max_diff_r2"], res["tsv_lines_differing"]))


# ------------------------------------------------------------ dense, bit for bit
@pytest.mark.parametrize("L,N,seed", [(2, 7, 0), (40, 1, 1), (40, 3, 2), (37, 8, 3), (64, 9, 4), (70, 15, 5),
                                      (65, 16, 6), (66, 17, 7), (130, 129, 8), (300, 500, 9), (257, 1000, 10),
                                      (120, 2001, 11), (90, 5008, 12)])
def test_ref_dense_bit_exact_synthetic(ref_ctx, L, N, seed):
    # every N mod 8 (the scalar tail), N < 8 (no lane loop at all), lane
    # classes longer than one 64-sequence stage, one- and many-stage classes
    buf = synth(L, N, seed)
    rng = np.random.default_rng(seed + 100)
    for w in (rng.random(N).astype(np.float32), np.ones(N, dtype=np.float32),
              (2.0 ** rng.uniform(-12, 0, N)).astype(np.float32)):
        ref_ctx.load(buf, w)
        assert_dense_bit_exact(ref_ctx, buf, w)


def test_ref_dense_mixed_sign_and_awkward_sites(ref_ctx):
    rng = np.random.default_rng(9)
    L, N = 90, 77
    buf = rng.choice(6, size=(L, N), p=[0.3, 0.3, 0.1, 0.1, 0.1, 0.1]).astype(np.uint8)
    buf[0] = 0
    buf[1] = 5
    buf[2] = np.where(np.arange(N) % 2, 0, 4)
    buf[3] = np.where(np.arange(N) % 3 == 0, 1, 2)
    w = rng.random(N).astype(np.float32)
    w[::5] = 0.0
    ref_ctx.load(buf, w)
    assert_dense_bit_exact(ref_ctx, buf, w)
    w2 = (rng.random(N) - 0.3).astype(np.float32)  # signed weights: cancelling sums, same order -> same bits
    ref_ctx.load(buf, w2)
    assert_dense_bit_exact(ref_ctx, buf, w2)


def test_ref_dense_nonfinite_weights(W):
    # non-finite weights: the select loop (0*inf must not appear) in lane-class order
    ctx = W.Context(0, W.KERNEL_VALU)
    ctx.set_option("ref_sums", 1)
    buf = synth(70, 45, 11)
    w = np.random.default_rng(3).random(45).astype(np.float32)
    w[5] = np.inf
    w[9] = np.nan
    w[44] = -np.inf  # in the scalar tail
    ctx.load(buf, w)
    assert_dense_bit_exact(ctx, buf, w)


def test_ref_known_answers(W, librs_ka):
    ctx = W.Context(0)
    ctx.set_option("ref_sums", 1)
    for c in librs_ka["ld_pair"]["cases"]:
        a, b = W.api.symbols_from_str(c["a"]), W.api.symbols_from_str(c["b"])
        wv = np.array(c["w"], dtype=np.float32)
        r = W.single_weighted_ld_pair(a, None, b, None, wv, ctx=ctx)
        o = O.single_pair(a, b, wv)
        assert r is not None and o is not None
        assert _bits_equal(np.array([r.d, r.d_prime, r.r2], np.float32), np.array(o, np.float32)).all(), (c["ref"], r, o)


# ------------------------------------------------- rows (behind the screen), bit for bit
def _cases():
    return ["random_henikoff", "ld_blocks", "rare_carriers", "mixed_sign", "vcf_like"]


def _make(W, case):
    if case == "random_henikoff":
        buf = synth(1500, 1000, 3)
        return buf, W.henikoff_weights(W.SiteSet.from_buffer(buf)), [0.0, 0.01, 0.05, 0.3]
    if case == "ld_blocks":
        buf = ld_blocks(1200, 800, 4)
        return buf, W.henikoff_weights(W.SiteSet.from_buffer(buf)), [0.05, 0.3, 0.8, 0.95]
    if case == "rare_carriers":
        buf, w = rare_carriers(900, 2000, 5)
        return buf, w, [0.0, 0.05, 0.1, 0.5]
    if case == "mixed_sign":
        buf = synth(700, 600, 6)
        rng = np.random.default_rng(7)
        w = (0.5 + 0.5 * rng.random(600)).astype(np.float32)
        neg = rng.random(600) < 0.1
        w[neg] = -(0.1 + 0.2 * rng.random(int(neg.sum()))).astype(np.float32)
        return buf, w, [0.01, 0.05, 0.2]
    buf = bench.vcf_like(2000, 5008, seed=77)
    return buf, W.henikoff_weights(W.SiteSet.from_buffer(buf)), [0.05, 0.1, 0.5]


@pytest.mark.parametrize("case", _cases())
def test_ref_rows_bit_exact(W, case):
    """Rows of the reference-order path equal the oracle's exactly (same
    rows, same order, same bits) behind the screen (forced one-plane,
    two-plane, auto) and without it."""
    buf, w, thrs = _make(W, case)
    ctx = W.Context(0, W.KERNEL_AUTO)
    ctx.set_option("ref_sums", 1)
    ctx.load(buf, w)
    screened = set()
    for thr in thrs:
        ref = O.all_pairs(buf, w, np.float32(thr))
        for screen in (1, 2, 3, 0):
            ctx.set_option("screen", screen)
            ctx.run(thr)
            st = ctx.stats()
            assert st["ref_sums"] == 1
            screened.add(st["screened"])
            assert_rows_bit_exact(ctx.rows(), ref)
        ctx.set_option("screen", 1)
    if ctx.stats()["kernel"] == W.KERNEL_MFMA:
        assert 1 in screened  # the i8 screen ran in front of the f32 reference-order kernel


# ----------------------------------------------------- the reports
def _report_set(W, name, buf, w, thrs):
    """Default path and reference-order path against the oracle (ordered and
    tree horizontal sums) at each threshold; one oracle run per order at the
    lowest threshold, the others are its strict-'>' subsets."""
    lo = np.float32(min(thrs))
    refs = {}
    for order in ("ordered", "tree"):
        with O.hsum_order(order):
            refs[order] = O.all_pairs(buf, w, lo)
    dflt = W.Context(0, W.KERNEL_AUTO, ref_sums=False)  # exact sums rounded once
    dflt.load(buf, w)
    refc = W.Context(0, W.KERNEL_AUTO)  # the default: lib.rs's order
    assert refc.get_option("ref_sums") == 1
    refc.load(buf, w)
    out = {}
    for thr in thrs:
        t32 = np.float32(thr)
        sub = {k: {f: v[f][v["r2"] > t32] for f in ("site_a", "site_b", "d", "d_prime", "r2")}
               for k, v in refs.items()}
        dflt.run(thr)
        d_rows = dflt.rows()
        refc.run(thr)
        r_rows = refc.rows()
        for mode, rows in (("exact", d_rows), ("ref_sums", r_rows)):
            for order in ("ordered", "tree"):
                res = row_diff(rows, sub[order], thr)
                out[(thr, mode, order)] = res
                REF_REPORT.append(_fmt("%s thr %g" % (name, thr), "%s vs %s" % (mode, order), res))
        assert_rows_bit_exact(r_rows, sub["ordered"])
    return out


def test_report_rare_and_vcf_like(W):
    buf, w = rare_carriers(900, 2000, 5)
    _report_set(W, "rare_carriers 900x2000", buf, w, [0.05, 0.1])
    buf = bench.vcf_like(3000, 5008)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    _report_set(W, "vcf_like 3000x5008 Henikoff", buf, w, [0.05, 0.1])


@pytest.mark.parametrize("cfg", ["c4", "c5"])
def test_report_full_bench_workloads(W, cfg):
    """BASELINE configs 4 and 5 at full size (the bench's own seeded inputs,
    Henikoff weights): every row of the GPU paths against the oracle over the
    whole pair space (about 5 s / 30 s of oracle on 16 threads), at the bench
    threshold 0.05 and at a low threshold that emits rows on random data:
    0.01 at C4 (~1,500 rows), 0.003 at C5 (~10^5 rows: N r2 = 15 is the
    chi-square tail the null pairs of 5,000 sequences reach)."""
    N, L, thr, _ = bench.CONFIGS[cfg]
    buf = bench.synth(L, N)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    lo = np.float32(0.01 if cfg == "c4" else 0.003)
    ref = O.all_pairs(buf, w, lo)
    assert ref["pairs"] == L * (L - 1) // 2
    assert len(ref["r2"]) > (1000 if cfg == "c4" else 50000), len(ref["r2"])
    for mode in ("exact", "ref_sums"):
        ctx = W.Context(0, W.KERNEL_AUTO, ref_sums=mode == "ref_sums")
        ctx.load(buf, w)
        for t in (thr, float(lo)):
            t32 = np.float32(t)
            sub = {f: v[ref["r2"] > t32] for f, v in ref.items() if f != "pairs"}
            ctx.run(t)
            rows = ctx.rows()
            res = row_diff(rows, sub, t)
            REF_REPORT.append(_fmt("%s full %dx%d thr %g" % (cfg, N, L, t), "%s vs ordered" % mode, res))
            if mode == "ref_sums":
                assert_rows_bit_exact(rows, sub)
            else:
                # exact sums rounded once: rows may differ only on the cut
                assert res["one_sided_outside_band"] == 0, res
                assert res["beyond_tol_d"] == 0 and res["beyond_tol_r2"] == 0, res
        ctx.close()


def test_c5_ldblocks_rows_bit_exact(W):
    """BASELINE config 5's size with linkage blocks (bench --data ldblocks at
    5,000 x 50,000): at the bench threshold 0.05 hundreds of thousands of rows
    pass — the screen's candidate tiles, staging, the chunk scan and the
    reference-order gather at 1.25e9 pairs — and every row equals the
    oracle's, bit for bit and in order (the default, lib.rs's order)."""
    N, L, thr, _ = bench.CONFIGS["c5"]
    buf = bench.ld_blocks(L, N)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    ref = O.all_pairs(buf, w, np.float32(thr))
    assert len(ref["r2"]) > 100000, len(ref["r2"])
    ctx = W.Context(0, W.KERNEL_AUTO)
    ctx.load(buf, w)
    n = ctx.run(thr)
    REF_REPORT.append("c5 ldblocks %dx%d thr %g: rows %d (oracle %d), screened %d" % (
        N, L, thr, n, len(ref["r2"]), ctx.stats()["screened"]))
    assert_rows_bit_exact(ctx.rows(), {f: v for f, v in ref.items() if f != "pairs"})
    ctx.close()


def test_ref_screen_policy(W):
    # lib.rs's order, auto policy: the one-plane screen until it leaves more
    # than half the tiles as candidates; then the exact candidate pairs, each
    # summed alone (screened 4), until those are more than a tenth of all
    # pairs; then the full f32 kernel.  Rows bit-identical to the oracle at
    # every step of the policy.
    ctx = W.Context(0, W.KERNEL_AUTO)
    ctx.set_option("screen_fp6", 0)  # the i8 tiers (test_gpu_fp6.py: the fp6 screen's handover)
    buf = synth(2000, 2000, 23)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    ctx.load(buf, w)
    seen = []
    for thr in (0.002, 0.002, 0.002, 0.003, 0.0005, 0.0005, 0.05):
        n = ctx.run(thr)
        st = ctx.stats()
        seen.append((thr, st["screened"], st["candidate_tiles"], st["tiles"], st["candidate_pairs"], st["pairs"]))
        assert n == len(ctx.rows())
        assert_rows_bit_exact(ctx.rows(), O.all_pairs(buf, w, np.float32(thr)))
    assert seen[0][1] == 1, seen
    for prev, cur in zip(seen[:5], seen[1:6]):
        if cur[0] > prev[0]:
            continue  # a higher threshold may screen again
        if prev[1] == 1:
            assert cur[1] == (4 if prev[2] * 2 > prev[3] else 1), seen
        elif prev[1] == 4:
            assert cur[1] == (0 if prev[4] * 10 > prev[5] else 4), seen
            assert prev[4] >= n  # the candidates include every row
    assert seen[-1][1] == 1, seen


@pytest.mark.parametrize("case", ["random", "ldblocks", "rare", "mixed_sign"])
@pytest.mark.parametrize("thr", [0.002, 0.01, 0.05])
def test_ref_pairs_rows_bit_exact(W, case, thr):
    # WLD_OPT_SCREEN 4: every tile on all i8 planes, the pairs the bound cannot
    # reject (the reference's rounding as residual) summed one by one in
    # lib.rs's order: the rows (order, indices, d, d', r2) are the oracle's bit
    # for bit, and every row was a candidate.
    rng = np.random.default_rng(7)
    w = None
    if case == "random":
        buf = synth(700, 300, 17)
    elif case == "ldblocks":
        buf = ld_blocks(900, 257, 3)
    elif case == "rare":
        buf, w = rare_carriers(600, 301, 5)
    else:
        buf = synth(500, 203, 19)
    if w is None:
        w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    if case == "mixed_sign":
        w = (rng.random(buf.shape[1]) - 0.3).astype(np.float32)
    ctx = W.Context(0, W.KERNEL_AUTO)
    ctx.set_option("screen", 4)
    ctx.load(buf, w)
    n = ctx.run(thr)
    st = ctx.stats()
    ref = O.all_pairs(buf, w, np.float32(thr))
    if st["kernel"] == W.KERNEL_MFMA:
        assert st["screened"] == 4 and st["candidate_pairs"] >= n, st
    assert_rows_bit_exact(ctx.rows(), ref)


def test_ref_pairs_staging_regrow(W):
    # a staging overflow of the candidate rows re-runs the pass with enough
    # staging: the same rows
    buf = synth(800, 300, 29)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    ctx = W.Context(0, W.KERNEL_AUTO)
    ctx.set_option("screen", 4)
    ctx.set_option("staging_rows", 64)
    ctx.load(buf, w)
    n = ctx.run(0.003)
    assert ctx.stats()["screened"] == 4 and n > 64
    assert_rows_bit_exact(ctx.rows(), O.all_pairs(buf, w, np.float32(0.003)))


def test_modes_and_tiers_on_one_context(W):
    # One context switched between lib.rs's order and the exact mode and across
    # every tier (screen + candidate tiles, candidate pairs, full kernel, the
    # two-plane screen of the exact mode): lib.rs-order rows bit-identical to
    # the oracle each time, exact-mode rows the same set with values within
    # 1e-5 (or closer to the f64 truth), no state leaking between runs.
    from test_gpu_parity import compare_rows
    buf = ld_blocks(1200, 301, 11)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    ctx = W.Context(0, W.KERNEL_AUTO)
    ctx.load(buf, w)
    plan = [(1, 1, 0.05), (1, 4, 0.003), (0, 1, 0.003), (1, 1, 0.003), (0, 3, 0.01), (1, 0, 0.05),
            (1, 2, 0.02), (0, 1, 0.05), (1, 1, 0.0), (1, 4, 0.05)]
    for ref_sums, screen, thr in plan:
        ctx.set_option("ref_sums", ref_sums)
        ctx.set_option("screen", screen)
        n = ctx.run(thr)
        ref = O.all_pairs(buf, w, np.float32(thr))
        if ref_sums:
            assert_rows_bit_exact(ctx.rows(), ref)
        else:
            compare_rows(ctx.rows(), ref, np.float32(thr), buf=buf, w=w)
        assert n == len(ctx.rows())
