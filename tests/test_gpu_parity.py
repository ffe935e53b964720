"""GPU parity tests: the HIP path through the C ABI against the CPU oracle.

Tolerance: north_star — D, D' and r2 within 1e-5 (f32).  Row sets must match
exactly except for rows whose r2 lies within 1e-5 of the threshold (a strict
'>' on floating point sums computed in a different order), and the rows must
come in the reference order (triu chunk order, then a, then b).
"""
import math
import os
import re
import subprocess

import numpy as np
import pytest

import _oracle as O
from conftest import CLI, FIXTURES, REPO, SYNTH

pytestmark = pytest.mark.gpu

TOL = 1e-5
# "valu" / "mfma": the f32 kernel's two-level sums and the integer MFMA
# kernel's exact sums (WLD_OPT_REF_SUMS 0); "ref": the default, lib.rs's own
# f32 summation order (bit-identical to the oracle; within TOL a fortiori)
KERNELS = ["valu", "mfma", "ref"]


@pytest.fixture(scope="module")
def W():
    import weightedld_amd as W
    return W


@pytest.fixture(scope="module")
def ctxs(W):
    out = {"valu": W.Context(0, W.KERNEL_VALU, ref_sums=False)}
    if W.lib().wld_set_kernel(out["valu"]._h, W.KERNEL_MFMA) == 0:
        out["mfma"] = W.Context(0, W.KERNEL_MFMA, ref_sums=False)
    out["valu"].set_kernel(W.KERNEL_VALU)
    out["ref"] = W.Context(0)
    return out


def new_ctx(W, kern, **kw):
    """A fresh context of the same kind as ctxs[kern]."""
    if kern == "ref":
        return W.Context(0, **kw)
    return W.Context(0, W.KERNEL_MFMA if kern == "mfma" else W.KERNEL_VALU, ref_sums=False, **kw)


def _ctx(ctxs, kern):
    if kern not in ctxs:
        pytest.skip("%s kernel not built" % kern)
    return ctxs[kern]


def sys_path_bench():
    import sys
    if REPO not in sys.path:
        sys.path.insert(0, REPO)


def synth(L, N, seed, p_missing=0.1, p_major=0.6, unknown=0.0):
    """bench_weighted_pair_ld.rs:8-28 distribution, seeded."""
    rng = np.random.default_rng(seed)
    maj = rng.integers(0, 4, size=L)
    mnr = (maj + rng.integers(1, 4, size=L)) % 4
    u = rng.random((L, N))
    codes = np.where(u < p_missing, 4, np.where(u < p_missing + p_major, maj[:, None], mnr[:, None]))
    if unknown:
        codes = np.where(rng.random((L, N)) < unknown, 5, codes)
    return codes.astype(np.uint8)


def agree(g, r, t=None, tol=TOL, field=None, escape=None, den=None):
    """Per-value parity criterion.  g: GPU f32, r: oracle f32 (lib.rs
    semantics), t: f64 value of the same sums/epilogue (or None).
    Strict: within tol of the reference (relative for |r| > 1, where f32 itself
    has no 1e-5 absolute resolution); NaN/inf must match.  d and r2 must pass
    strictly.  D' alone (field "d_prime") may instead be no farther from the
    exact value t than twice the f32 reference's own error (+1e-6): both run
    the same f32 epilogue (lib.rs:482-520), whose cancellations D' = D/den
    amplifies when den is small, on differently rounded sums (the reference's
    8-lane f32 sums, ~N/8 * 2^-24 relative; the GPU's exact sums rounded
    once), so on such pairs each is off the exact value by epilogue noise of
    the same size.  That noise is a few f32 ulps of the 2x2 cell terms over
    den = |d / D'| (the exact values): with den given, D' may also be within
    8 * 2^-24 / den of t (the reference itself reaches 4.7 such units on the
    clustered set of test_gpu_screen, and f32 epilogues on the exactly
    rounded, unquantised sums 3.1).  escape=True extends the escape to every
    field (only for inputs outside the reference's own 1e-5 accuracy, e.g.
    minor alleles carried by a few low-weight sequences).  Every escape is
    counted, with its |GPU - reference|, in the session's parity report
    (conftest.py)."""
    from conftest import PARITY
    g = np.asarray(g, dtype=np.float64)
    r = np.asarray(r, dtype=np.float64)
    with np.errstate(invalid="ignore"):
        special = (np.isnan(g) & np.isnan(r)) | (np.isinf(g) & np.isinf(r) & (np.sign(g) == np.sign(r)))
        diff = np.abs(g - r)
        strict = special | (diff <= tol * np.maximum(1.0, np.abs(r)))
        ok = strict.copy()
        esc = np.zeros_like(ok)
        if escape is None:
            escape = field == "d_prime"
        if t is not None and escape:
            t = np.asarray(t, dtype=np.float64)
            allow = 2.0 * np.abs(r - t)
            if den is not None:
                allow = np.maximum(allow, 8.0 * 2.0 ** -24 / np.asarray(den, dtype=np.float64))
            esc = ~strict & np.isfinite(t) & (np.abs(g - t) <= allow + 1e-6 * np.maximum(1.0, np.abs(t)))
            ok |= esc
        fin = strict & ~special
        PARITY.record(field or "value", len(g), float(diff[fin].max()) if fin.any() else 0.0,
                      int(esc.sum()), float(diff[esc].max()) if esc.any() else 0.0)
    return ok


def close(x, y, tol=TOL):
    return agree(x, y, None, tol)


def compare_dense(gpu, ref, truth=None, tol=TOL, mask=None):
    """mask (over the upper-triangle pairs, optional): compare only those."""
    d, dp, r2, valid = gpu
    rd, rdp, rr2, rvalid = ref
    L = d.shape[0]
    iu = np.triu_indices(L, 1)
    assert np.array_equal(valid[iu], rvalid[iu])
    m = rvalid[iu] == 1
    if mask is not None:
        m &= mask
    den = None
    if truth is not None:
        with np.errstate(all="ignore"):
            den = np.abs(truth[0][iu][m] / truth[1][iu][m])
    for k, (g, r) in enumerate(((d, rd), (dp, rdp), (r2, rr2))):
        t = truth[k][iu][m] if truth is not None else None
        ok = agree(g[iu][m], r[iu][m], t, tol, ("d", "d_prime", "r2")[k], den=den if k == 1 else None)
        assert ok.all(), ("dsr"[k], np.count_nonzero(~ok), g[iu][m][~ok][:5], r[iu][m][~ok][:5],
                          None if t is None else t[~ok][:5])


def dense_check(ctx, buf, w):
    L = buf.shape[0]
    compare_dense(ctx.dense(L), O.all_pairs_dense(buf, w), O.all_pairs_dense_f64(buf, w)[:3])


def compare_rows(store, ref, thr, tol=TOL, buf=None, w=None, site_map=None):
    ka = list(zip(store.site_a.tolist(), store.site_b.tolist()))
    kb = list(zip(ref["site_a"].tolist(), ref["site_b"].tolist()))
    ga = {k: i for i, k in enumerate(ka)}
    gb = {k: i for i, k in enumerate(kb)}
    assert len(ga) == len(ka), "duplicate rows"
    only_gpu = [k for k in ka if k not in gb]
    only_ref = [k for k in kb if k not in ga]
    for k in only_gpu:
        assert abs(store.r2[ga[k]] - thr) <= tol, ("extra row", k, store.r2[ga[k]])
    for k in only_ref:
        assert abs(ref["r2"][gb[k]] - thr) <= tol, ("missing row", k, ref["r2"][gb[k]])
    common = [k for k in ka if k in gb]
    # same relative order
    assert [k for k in kb if k in ga] == common
    ia = np.array([ga[k] for k in common], dtype=np.int64)
    ib = np.array([gb[k] for k in common], dtype=np.int64)
    if len(common):
        truth = [None, None, None]
        if buf is not None:
            td, tdp, tr2, _ = O.all_pairs_dense_f64(buf, w)
            inv = {int(p): i for i, p in enumerate(site_map)} if site_map is not None else None
            fa = np.array([inv[a] if inv else a for a, _ in common])
            fb = np.array([inv[b] if inv else b for _, b in common])
            truth = [td[fa, fb], tdp[fa, fb], tr2[fa, fb]]
        den = None
        if truth[0] is not None:
            with np.errstate(all="ignore"):
                den = np.abs(truth[0] / truth[1])
        for k, f in enumerate(("d", "d_prime", "r2")):
            ok = agree(getattr(store, f)[ia], ref[f][ib], truth[k], tol, f, den=den if k == 1 else None)
            assert ok.all(), (f, np.count_nonzero(~ok), getattr(store, f)[ia][~ok][:5], ref[f][ib][~ok][:5],
                              None if truth[k] is None else truth[k][~ok][:5])
    return len(common), len(only_gpu), len(only_ref)


# ------------------------------------------------------------------ known answers
def test_librs_known_answers_on_gpu(W, librs_ka):
    for c in librs_ka["ld_pair"]["cases"]:
        r = W.single_weighted_ld_pair(W.api.symbols_from_str(c["a"]), None, W.api.symbols_from_str(c["b"]), None,
                                      np.array(c["w"], dtype=np.float32))
        assert r is not None
        assert abs(r.d - c["d"]) <= c["tol"] and abs(r.d_prime - c["d_prime"]) <= c["tol"] and abs(r.r2 - c["r2"]) <= c["tol"], (c["ref"], r)
    assert W.single_weighted_ld_pair(W.api.symbols_from_str("AAAAAAAA"), None, W.api.symbols_from_str("ACACACAC"),
                                     None, np.ones(8, dtype=np.float32)) is None


# ------------------------------------------------------------------ dense parity
@pytest.mark.parametrize("kern", KERNELS)
@pytest.mark.parametrize("L,N,seed", [(2, 7, 0), (37, 50, 1), (64, 64, 2), (130, 129, 3), (300, 500, 4), (257, 1000, 5)])
def test_dense_vs_oracle_synthetic(ctxs, kern, L, N, seed):
    ctx = _ctx(ctxs, kern)
    buf = synth(L, N, seed)
    w = np.random.default_rng(seed + 100).random(N).astype(np.float32)
    for weights in (w, np.ones(N, dtype=np.float32)):
        ctx.load(buf, weights)
        dense_check(ctx, buf, weights)


@pytest.mark.parametrize("kern", KERNELS)
def test_dense_vs_oracle_awkward_sites(ctxs, kern):
    # monomorphic (None), all-Unknown, Missing as minor, ties, Unknown sprinkled
    ctx = _ctx(ctxs, kern)
    rng = np.random.default_rng(9)
    L, N = 90, 77
    buf = rng.choice(6, size=(L, N), p=[0.3, 0.3, 0.1, 0.1, 0.1, 0.1]).astype(np.uint8)
    buf[0] = 0
    buf[1] = 5
    buf[2] = np.where(np.arange(N) % 2, 0, 4)
    buf[3] = np.where(np.arange(N) % 3 == 0, 1, 2)
    w = rng.random(N).astype(np.float32)
    w[::5] = 0.0
    ctx.load(buf, w)
    dense_check(ctx, buf, w)


@pytest.mark.parametrize("kern", KERNELS)
@pytest.mark.parametrize("N", [1, 2, 3])
def test_dense_vs_oracle_few_sequences(ctxs, kern, N):
    # one to three sequences (63 padding lanes of the 64-sequence step): masks
    # of one or two sequences, T = a single weight, 0/0 NaN rows
    ctx = _ctx(ctxs, kern)
    rng = np.random.default_rng(N)
    buf = rng.choice(5, size=(40, N)).astype(np.uint8)
    w = (0.3 + rng.random(N)).astype(np.float32)
    ctx.load(buf, w)
    dense_check(ctx, buf, w)
    ctx.run(0.0)
    compare_rows(ctx.rows(), O.all_pairs(buf, w, 0.0), 0.0, buf=buf, w=w)


def test_dense_nonfinite_weights_valu(ctxs):
    # non-finite weights force the SAFE select variant (0*inf must not appear)
    ctx = ctxs["valu"]
    buf = synth(70, 40, 11)
    w = np.random.default_rng(3).random(40).astype(np.float32)
    w[5] = np.inf
    w[9] = np.nan
    ctx.load(buf, w)
    dense_check(ctx, buf, w)


@pytest.mark.parametrize("kern", KERNELS)
def test_dense_vs_oracle_many_sequences(ctxs, kern):
    # BASELINE config 5's sequence count: 5000 -> 158 32-sequence stages,
    # 20 LDS groups with a partial last group
    ctx = _ctx(ctxs, kern)
    buf = synth(150, 5000, 21)
    import weightedld_amd as W
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    ctx.load(buf, w)
    dense_check(ctx, buf, w)


@pytest.mark.parametrize("kern", KERNELS)
def test_dense_vs_oracle_wide_sums(ctxs, kern):
    # 66,000 sequences: NP > 65024, so the MFMA epilogue takes the wide form
    # (S = acc0 + 2^8 acc1 + 2^16 acc2 assembled in f64, no int32 pre-combination)
    ctx = _ctx(ctxs, kern)
    buf = synth(40, 66000, 31)
    import weightedld_amd as W
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    ctx.load(buf, w)
    dense_check(ctx, buf, w)


@pytest.mark.parametrize("kern", KERNELS)
def test_dense_mixed_sign_weights(ctxs, kern):
    # Weights are any finite f32 in lib.rs; the MFMA fixed point is signed
    # (negative balanced digits).  ~10% small negative weights keep the sums
    # well-conditioned.  (With sums that cancel to ~0, D ~ 1/T^2 amplifies any
    # f32 or fixed-point rounding and no two summation orders agree to 1e-5 —
    # the reference's 8-lane f32 sums included)
    ctx = _ctx(ctxs, kern)
    buf = synth(120, 333, 17)
    rng = np.random.default_rng(9)
    w = (0.5 + 0.5 * rng.random(333)).astype(np.float32)
    neg = rng.random(333) < 0.1
    w[neg] = -(0.1 + 0.2 * rng.random(int(neg.sum()))).astype(np.float32)
    ctx.load(buf, w)
    dense_check(ctx, buf, w)


def test_auto_kernel_choice(W):
    # AUTO: MFMA for Henikoff-like weights, VALU when the dynamic range exceeds
    # 2^12 (4-plane fixed point could lose small weights) or a weight is non-finite
    buf = synth(200, 100, 23)
    ctx = W.Context(0, W.KERNEL_AUTO)
    w = np.random.default_rng(1).random(100).astype(np.float32) + 0.5
    ctx.load(buf, w)
    assert ctx.stats()["kernel"] == W.KERNEL_MFMA
    w2 = w.copy()
    w2[3] = 1e-6
    ctx.load(buf, w2)
    assert ctx.stats()["kernel"] == W.KERNEL_VALU
    ctx.run(0.0)
    compare_rows(ctx.rows(), O.all_pairs(buf, w2, 0.0), 0.0, buf=buf, w=w2)
    w3 = w.copy()
    w3[7] = np.inf
    ctx.load(buf, w3)
    assert ctx.stats()["kernel"] == W.KERNEL_VALU


# ------------------------------------------------------- skipped weight-digit planes
# weights -> digit planes the MFMA kernel multiplies.  max|w| = 1 gives the
# fixed point q = rint(w 2^22) = d0 + 256 d1 + 65536 d2 (balanced digits):
# w = 1 -> d2 = 64 only; 3/256 -> d1 = -64, d2 = 1; 1 - 2^-22 -> d0 = -1, d2 = 64.
PLANE_CASES = {
    "unweighted": (lambda r, n: np.ones(n, np.float32), 1),
    "planes_1_2": (lambda r, n: np.where(r.random(n) < 0.5, 1.0, 3 / 256).astype(np.float32), 2),
    "planes_0_2": (lambda r, n: np.where(r.random(n) < 0.5, 1.0, 1.0 - 2.0 ** -22).astype(np.float32), 2),
    "henikoff_like": (lambda r, n: (0.2 + 0.8 * r.random(n)).astype(np.float32), 3),
    # a range beyond 2^-4: 4 planes (31-bit fixed point, q = rint(w 2^30) for max 1)
    "wide_4planes": (lambda r, n: np.where(r.random(n) < 0.5, 1.0, 0.01 + 0.02 * r.random(n)).astype(np.float32), 4),
    # (explicit MFMA) 4-plane shift, planes 3 and 1 only: q = rint(w 2^30):
    # w = 1 -> d3 = 64; w = 2^-16 -> d1 = 64
    "planes_1_3": (lambda r, n: np.where(r.random(n) < 0.5, 1.0, 2.0 ** -16).astype(np.float32), 2),
}


@pytest.mark.parametrize("case", sorted(PLANE_CASES))
def test_mfma_skips_zero_digit_planes(ctxs, case):
    # The kernel multiplies only the planes with a nonzero digit (4 products
    # each); the integer sums are the same, so every output is bit-identical
    # to the all-planes run (WLD_OPT_ALL_PLANES) and agrees with the oracle.
    ctx = _ctx(ctxs, "mfma")
    make_w, planes = PLANE_CASES[case]
    buf = synth(300, 700, 31)
    w = make_w(np.random.default_rng(5), 700)
    ctx.load(buf, w)
    assert ctx.stats()["mfma_planes"] == planes
    got = ctx.dense(300)
    compare_dense(got, O.all_pairs_dense(buf, w), O.all_pairs_dense_f64(buf, w)[:3])
    n = ctx.run(0.02)
    rows = ctx.rows()
    compare_rows(rows, O.all_pairs(buf, w, 0.02), 0.02, buf=buf, w=w)
    ctx.set_option("all_planes", 1)
    try:
        ctx.load(buf, w)
        # fixed point: 3 digit planes while min/max >= 2^-4, else 4
        nz = np.abs(w[w != 0])
        assert ctx.stats()["mfma_planes"] == (3 if nz.min() >= nz.max() * 2.0 ** -4 else 4)
        full = ctx.dense(300)
        iu = np.triu_indices(300, 1)
        for g, f in zip(got, full):
            assert np.array_equal(g[iu].view(np.uint32) if g.dtype == np.float32 else g[iu],
                                  f[iu].view(np.uint32) if f.dtype == np.float32 else f[iu])
        assert ctx.run(0.02) == n
    finally:
        ctx.set_option("all_planes", 0)


# ------------------------------------------------------------------ ordered rows
@pytest.mark.parametrize("kern", KERNELS)
@pytest.mark.parametrize("L,N,thr", [(1, 10, 0.0), (2, 10, 0.0), (255, 64, 0.0), (256, 100, 0.05), (257, 100, 0.0),
                                     (700, 300, 0.0), (700, 300, 0.01), (1100, 200, -1.0), (900, 2000, 0.001)])
def test_rows_vs_oracle(ctxs, kern, L, N, thr):
    ctx = _ctx(ctxs, kern)
    buf = synth(L, N, L * 7 + N)
    w = np.random.default_rng(L).random(N).astype(np.float32) + 0.05
    site_map = np.arange(L, dtype=np.uint64) * 3 + 11
    ctx.load(buf, w, site_map)
    n = ctx.run(thr)
    store = ctx.rows()
    assert len(store) == n
    ref = O.all_pairs(buf, w, thr, site_map=site_map)
    compare_rows(store, ref, thr, buf=buf, w=w, site_map=site_map)
    st = ctx.stats()
    assert st["pairs"] == L * (L - 1) // 2


@pytest.mark.parametrize("kern", KERNELS)
def test_staging_overflow_regrows(W, ctxs, kern):
    # staging starts tiny, the run detects the overflow from the cursor and re-runs
    _ctx(ctxs, kern)
    ctx = new_ctx(W, kern)  # fresh: no grown staging
    ctx.set_option("staging_rows", 100)
    L, N = 700, 150
    buf = synth(L, N, 5)
    w = np.random.default_rng(2).random(N).astype(np.float32)
    ctx.load(buf, w)
    n = ctx.run(0.0)
    assert n > 1000
    compare_rows(ctx.rows(), O.all_pairs(buf, w, 0.0), 0.0, buf=buf, w=w)


@pytest.mark.parametrize("kern", KERNELS)
def test_gather_behind_scan_sequences(W, ctxs, kern):
    """After a run with rows the gather is enqueued behind the scan before the
    host sees the row count (capi.hip enqueue_pass, WLD_SPEC_GATHER), with
    outputs for 1.25x the last run's rows.  Every case of that guess: more rows
    (gathered again into larger outputs), a staging overflow (the pass re-runs,
    the gather with it), no rows, fewer rows, a shard, a site map — each run's
    rows equal the oracle's."""
    _ctx(ctxs, kern)
    ctx = new_ctx(W, kern)
    ctx.set_option("staging_rows", 100)
    L, N = 700, 150
    buf = synth(L, N, 6)
    w = np.random.default_rng(3).random(N).astype(np.float32)
    ctx.load(buf, w)
    seq = [(0.5, None), (0.2, None), (0.0, None), (0.0, None), (1.01, None), (0.3, None), (0.0, (3,)), (0.1, None)]
    for thr, shard in seq:
        if shard:  # every shard of an n-way split: the full run's rows with a in its chunk rows
            full = O.all_pairs(buf, w, np.float32(thr))
            total = 0
            for k in range(shard[0]):
                b, e = ctx.shard_chunk_rows(L, shard[0], k)
                n = ctx.run(thr, b, e)
                sel = (full["site_a"] // 256 >= b) & (full["site_a"] // 256 < e)
                ref = {f: np.asarray(full[f])[sel] for f in ("site_a", "site_b", "d", "d_prime", "r2")}
                assert n == int(sel.sum())
                compare_rows(ctx.rows(), ref, thr, buf=buf, w=w)
                total += n
            assert total == len(full["site_a"]) > 0
            continue
        n = ctx.run(thr)
        ref = O.all_pairs(buf, w, np.float32(thr))
        assert n == len(ref["site_a"]), (thr, n)
        compare_rows(ctx.rows(), ref, thr, buf=buf, w=w)
    keep = np.arange(L, dtype=np.uint64) * 3 + 7
    ctx.load(buf, w, keep)
    for thr in (0.2, 0.2, 0.0):
        n = ctx.run(thr)
        ref = O.all_pairs(buf, w, np.float32(thr), site_map=keep)
        assert n == len(ref["site_a"])
        compare_rows(ctx.rows(), ref, thr, buf=buf, w=w, site_map=keep)
    ctx.close()


@pytest.mark.parametrize("kern", KERNELS)
@pytest.mark.parametrize("G", [2, 3, 4])
def test_sharded_runs_concatenate_to_reference_order(ctxs, kern, G):
    ctx = _ctx(ctxs, kern)
    L, N = 1500, 200
    buf = synth(L, N, 77)
    w = np.random.default_rng(1).random(N).astype(np.float32)
    ctx.load(buf, w)
    ctx.run(0.0)
    full = ctx.rows()
    parts = []
    for g in range(G):
        b, e = ctx.shard_chunk_rows(L, G, g)
        ctx.run(0.0, b, e)
        parts.append(ctx.rows())
    # chunk rows descend in reference order: shard G-1 comes first
    cat = lambda f: np.concatenate([getattr(p, f) for p in reversed(parts)])  # noqa: E731
    for f in ("site_a", "site_b", "d", "d_prime", "r2"):
        assert np.array_equal(cat(f), getattr(full, f)), f
    # the finer chunk-range shards (wld_shard_chunks / wld_run_chunks), which
    # split chunk rows mid-row, concatenate the same way
    parts = []
    for g in range(G):
        b, e = ctx.shard_chunks(L, G, g)
        assert ctx.run_chunks(0.0, b, e) == len(ctx.rows().site_a)
        assert ctx.stats()["pairs"] == ctx.pairs_in_chunks(L, b, e)
        parts.append(ctx.rows())
    for f in ("site_a", "site_b", "d", "d_prime", "r2"):
        assert np.array_equal(cat(f), getattr(full, f)), f


@pytest.mark.parametrize("kern", ["mfma", "valu"])
def test_single_chunk_runs_match_oracle(ctxs, kern):
    """Every chunk run alone (wld_run_chunks(i, i+1)) against the oracle's chunk range."""
    ctx = _ctx(ctxs, kern)
    L, N = 700, 96
    buf = synth(L, N, 5)
    w = np.random.default_rng(3).random(N).astype(np.float32)
    ctx.load(buf, w)
    for i in range(ctx.chunks(L)):
        ctx.run_chunks(0.0, i, i + 1)
        got = ctx.rows()
        ref = O.all_pairs(buf, w, 0.0, chunk_lo=i, chunk_hi=i + 1)
        assert np.array_equal(got.site_a, ref["site_a"].astype(np.uint32)), i
        assert np.array_equal(got.site_b, ref["site_b"].astype(np.uint32)), i
        for f in ("d", "d_prime", "r2"):
            np.testing.assert_allclose(getattr(got, f), ref[f], atol=1e-5, rtol=0, err_msg="%s chunk %d" % (f, i))


# ------------------------------------------------------------------ API + CLI
def test_all_weighted_ld_pairs_api_on_fixture(W):
    ss = W.read_fasta(os.path.join(FIXTURES, "example.fasta"))
    f = ss.filter_sites_of_interest(0.8, 0.02, 0.5)
    w = W.henikoff_weights(f)
    seen = []
    store = W.all_weighted_ld_pairs(f, w, 0.1, progress_report=seen.append)
    rows = list(store)
    assert len(rows) == 1 and rows[0][:2] == (0, 1)
    assert "%.3f %.3f %.3f" % (rows[0][2].d, rows[0][2].d_prime, rows[0][2].r2) == "0.107 0.345 0.237"
    # lib.rs:584 then :670-674 for its one chunk: the counter before that chunk's add
    assert seen == [0, 0]


@pytest.mark.parametrize("name", ["synth_n200_l24.fasta", "synth_n500_l40.fasta", "synth_n2000_l30.fasta"])
def test_gpu_vs_python_reference_goldens(W, python_ref, name):
    g = python_ref[name]
    ss = W.read_fasta(os.path.join(SYNTH, name))
    f = ss.filter_sites_of_interest()
    w = W.henikoff_weights(f)
    for weights, key in ((w, "pairs_weighted"), (np.ones_like(w), "pairs_unweighted")):
        store = W.all_weighted_ld_pairs(f, weights, float("-inf"))
        got = {(a, b): (s.d, s.d_prime, s.r2) for a, b, s in store}
        for a, b, D, Dp, R2 in g[key]:
            d, dp, r2 = got[(a, b)]
            assert abs(d - D) <= TOL and abs(dp - Dp) <= TOL and abs(r2 - R2) <= TOL


def test_gpu_vcf_config3_vs_python(W, python_ref):
    g = python_ref["t7_1000genome.vcf"]
    ss = W.read_vcf(os.path.join(FIXTURES, "t7_1000genome.vcf"))
    w = W.henikoff_weights(ss)
    store = W.all_weighted_ld_pairs(ss, w, float("-inf"))
    got = {(a, b): (s.d, s.d_prime, s.r2) for a, b, s in store}
    assert len(g["pairs_weighted"]) == 10
    for a, b, D, Dp, R2 in g["pairs_weighted"]:
        d, dp, r2 = got[(a, b)]
        assert abs(d - D) <= TOL and abs(dp - Dp) <= TOL and abs(r2 - R2) <= TOL



def test_gpu_vcf_config3_unweighted_vs_python(W, python_ref):
    """BASELINE config 3's unweighted leg: the HIP path's rows on the t7 VCF
    with unit weights (main.rs:150-153) equal lib.rs's (the oracle, bit for
    bit: the default summation order), and Python's own rule on top of them —
    skip a pair when round(PA, 1) or round(PB, 1) is 1.0 over the sequences
    major or minor at both sites (WeightedLD.py:197-237) — leaves exactly what
    Python prints: the header alone (WeightedLD.py:176, tests/golden)."""
    g = python_ref["t7_1000genome.vcf"]
    ss = W.read_vcf(os.path.join(FIXTURES, "t7_1000genome.vcf"))
    buf, sm = ss.buffer, ss.site_map
    ones = np.ones(ss.n_seqs(), dtype=np.float32)
    store = W.all_weighted_ld_pairs(ss, ones, float("-inf"))
    ref = O.all_pairs(buf, ones, float("-inf"), site_map=sm)
    assert len(store) == len(ref["site_a"]) == 10
    assert np.array_equal(store.site_a.astype(np.uint64), ref["site_a"])
    assert np.array_equal(store.site_b.astype(np.uint64), ref["site_b"])
    for f in ("d", "d_prime", "r2"):
        assert np.array_equal(getattr(store, f).view(np.uint32), ref[f].view(np.uint32)), f
    idx = {int(p): i for i, p in enumerate(sm)}
    printed = []
    for a, b, d, dp, r2 in zip(store.site_a, store.site_b, store.d, store.d_prime, store.r2):
        x, y = buf[idx[int(a)]], buf[idx[int(b)]]
        keep = (x != 5) & (y != 5)  # WeightedLD.py:181-185: Unknown at either site dropped
        fr = []
        for col in (x[keep], y[keep]):
            vals, cnt = np.unique(col, return_counts=True)
            order = np.argsort(-cnt, kind="stable")
            fr.append((vals[order[0]], vals[order[1]] if len(vals) > 1 else None))
        (ma, na), (mb, nb) = fr
        tgt = keep.copy()
        tgt[keep] = ((x[keep] == ma) | (x[keep] == na)) & ((y[keep] == mb) | (y[keep] == nb))
        PA = np.mean(x[tgt] == ma)
        PB = np.mean(y[tgt] == mb)
        if round(PA, 1) == 1.0 or round(PB, 1) == 1.0:  # WeightedLD.py:234-237
            continue
        printed.append((int(a), int(b), float(d), float(dp), float(r2)))
    assert printed == g["pairs_unweighted"] == []


# expected Rust CLI output derived from lib.rs semantics
CLI_EXPECT = {
    ("example.fasta", False): ["0\t1\t0.107\t0.345\t0.237"],
    ("example.fasta", True): [],
    ("t2_henikoff_complex1.fasta", False): ["1\t2\t0.107\t0.357\t0.238"],
    ("t3_henikoff_complex2.fasta", False): ["1\t2\t0.107\t0.357\t0.238"],
    ("t4_weights1_ld0.fasta", False): ["0\t3\t0.088\t0.422\t0.192", "1\t3\t0.088\t0.422\t0.192"],
    ("t5_weights1_ld0.25.fasta", False): ["0\t1\t-0.250\t0.500\t1.000"],
    ("t5_weights1_ld0.25.fasta", True): ["0\t1\t-0.250\t0.500\t1.000"],
    ("t6_varsites_hk_ld.fasta", False): ["0\t1\t-0.148\t0.444\t0.400"],
    ("t6_varsites_hk_ld.fasta", True): ["0\t1\t-0.070\t0.700\t0.259"],
}


@pytest.mark.parametrize("case", sorted(CLI_EXPECT))
def test_cli_tsv(tmp_path, case):
    name, unweighted = case
    out = tmp_path / "pairs.tsv"
    cmd = [CLI, "--fasta-input", os.path.join(FIXTURES, name), "--pair-output", str(out)]
    if unweighted:
        cmd.append("--unweighted")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = out.read_text().splitlines()
    assert lines[0] == "site_a\tsite_b\td\td'\tr2"
    assert lines[1:] == CLI_EXPECT[case]
    assert "pairs computed at" in r.stderr


def test_cli_t1_panics_like_reference(tmp_path):
    r = subprocess.run([CLI, "--fasta-input", os.path.join(FIXTURES, "t1_henikoff_paper.fasta"), "--pair-output",
                        str(tmp_path / "p.tsv")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 101 and "panicked" in r.stderr


def test_cli_vcf_threshold_zero(tmp_path, python_ref):
    out = tmp_path / "pairs.tsv"
    r = subprocess.run([CLI, "--vcf-input", os.path.join(FIXTURES, "t7_1000genome.vcf"), "--pair-output", str(out),
                        "--r2-threshold", "0"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = out.read_text().splitlines()[1:]
    exp = ["%d\t%d\t%.3f\t%.3f\t%.3f" % (a, b, d, dp, r2) for a, b, d, dp, r2 in
           python_ref["t7_1000genome.vcf"]["pairs_weighted"]]
    assert sorted(lines) == sorted(exp)


# ------------------------------------------------------------------ full size (BASELINE config 4)
@pytest.mark.parametrize("kern", KERNELS)
def test_config4_full_size_properties(ctxs, kern):
    """N=2000 x L=20000, thr 0.05: size-independent properties plus a sampled
    oracle check (the oracle at full size takes minutes, a sample seconds)."""
    ctx = _ctx(ctxs, kern)
    L, N = 20000, 2000
    buf = synth(L, N, 2024)
    import weightedld_amd as W
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    ctx.load(buf, w)
    n = ctx.run(0.05)
    store = ctx.rows()
    st = ctx.stats()
    assert st["pairs"] == L * (L - 1) // 2 == 199990000
    assert len(store) == n
    if n:
        assert np.all(store.r2 > 0.05)
        assert np.all(store.site_a < store.site_b)
    # reference order of the emitted rows
    nchunk = (L + 255) // 256
    ca, cb = store.site_a.astype(np.int64) // 256, store.site_b.astype(np.int64) // 256
    rf = nchunk - 1 - ca
    lin = rf * (rf + 1) // 2 + (cb - ca)
    key = lin * (L * L) + store.site_a.astype(np.int64) * L + store.site_b
    assert np.all(np.diff(key) > 0)
    # sampled exact check against the oracle: a 600-site window at thr -inf
    sub = buf[9000:9600]
    ctx.load(sub, w)
    ctx.run(float("-inf"))
    compare_rows(ctx.rows(), O.all_pairs(sub, w, float("-inf")), float("-inf"), buf=sub, w=w)


def test_mfma_lds_pipeline_race_screen(W):
    """Race screen for the MFMA kernel's LDS pipeline (global_load_lds groups):
    the fragment-major LDS path and the site-major register path compute the
    same exact integer sums and the same f32 epilogue, so at config-4 size and
    a low threshold (~4e7 rows, 256-workgroup waves over every CU) they must
    agree bit for bit, run after run."""
    import torch
    from weightedld_amd import dist as wdist
    L, N = 20000, 2000
    buf = synth(L, N, 77)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    dev = torch.device("cuda", 0)
    # reference: the site-major register kernel, every pair through the f32
    # epilogue (no prefilter, no screen); under test: the LDS kernel behind the
    # one- and two-plane screens (at 0.001 nearly every tile is a candidate:
    # the looping candidate launch) with the prefilter
    ref_ctx = W.Context(0, W.KERNEL_MFMA, ref_sums=False)
    ref_ctx.set_option("prefilter", 0)
    ref_ctx.set_option("mfma_layout", 1)
    ref_ctx.load(buf, w)
    n_ref = ref_ctx.run(0.001)
    ref = wdist.pack_rows_device(ref_ctx, n_ref, dev)
    del ref_ctx
    ctx = W.Context(0, W.KERNEL_MFMA, ref_sums=False)
    ctx.load(buf, w)
    assert n_ref > 10_000_000
    # forced: auto would send 0.001 to the full kernel after the first run
    for mode, kind in ((2, 1), (3, 3), (2, 1), (3, 3)):
        ctx.set_option("screen", mode)
        n = ctx.run(0.001)
        assert n == n_ref
        assert ctx.stats()["screened"] == kind
        got = wdist.pack_rows_device(ctx, n, dev)
        assert torch.equal(got, ref)


def test_config5_full_size_properties(W):
    """BASELINE config 5 at one GPU: N=5000 x L=50000 (~1.25e9 pairs), thr 0.05.
    Size-independent properties of the emitted rows plus an exact oracle check
    of a 400-site window at thr -inf."""
    L, N = 50000, 5000
    buf = synth(L, N, 55)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    ctx = W.Context(0, W.KERNEL_MFMA)
    ctx.load(buf, w)
    n = ctx.run(0.05)
    st = ctx.stats()
    assert st["pairs"] == L * (L - 1) // 2
    store = ctx.rows()
    assert len(store) == n
    if n:
        assert np.all(store.r2 > 0.05)
        assert np.all(store.site_a < store.site_b)
        nchunk = (L + 255) // 256
        ca, cb = store.site_a.astype(np.int64) // 256, store.site_b.astype(np.int64) // 256
        rf = nchunk - 1 - ca
        lin = rf * (rf + 1) // 2 + (cb - ca)
        key = lin * (L * L) + store.site_a.astype(np.int64) * L + store.site_b
        assert np.all(np.diff(key) > 0)
    sub = buf[31000:31400]
    ctx.load(sub, w)
    ctx.run(float("-inf"))
    compare_rows(ctx.rows(), O.all_pairs(sub, w, float("-inf")), float("-inf"), buf=sub, w=w)


# ------------------------------------------------------------ async run + ShardStep
def test_run_chunks_async_matches_sync(W, ctxs):
    # wld_run_chunks_async + wld_run_wait == wld_run_chunks: same rows, the row
    # total in the caller's device word, the staging-regrow re-run inside
    # run_wait, and an empty range writing 0.
    import torch

    ctx = _ctx(ctxs, "mfma")
    L, N = 900, 300
    buf = synth(L, N, 77)
    w = np.random.default_rng(3).random(N).astype(np.float32) + 0.1
    ctx.load(buf, w)
    cnt = torch.full((1,), -1, dtype=torch.int64, device="cuda:0")
    for thr, init_rows in ((0.0, None), (0.01, None), (0.0, 1000)):
        if init_rows:
            ctx = W.Context(0, W.KERNEL_MFMA)  # fresh staging sized by the option
            ctx.set_option("staging_rows", init_rows)
            ctx.load(buf, w)
        ctx.run_chunks_async(thr, 0, 0, cnt.data_ptr())  # first: with tiny staging it must regrow
        n = ctx.run_wait()
        torch.cuda.synchronize()
        got = ctx.rows()
        n_ref = ctx.run_chunks(thr, 0, 0)
        ref = ctx.rows()
        assert n == n_ref == int(cnt.item())
        for f in ("site_a", "site_b", "d", "d_prime", "r2"):
            assert np.array_equal(getattr(got, f).view(np.uint32), getattr(ref, f).view(np.uint32)), f
    ctx.run_chunks_async(0.0, 3, 3, cnt.data_ptr())
    assert ctx.run_wait() == 0
    torch.cuda.synchronize()
    assert int(cnt.item()) == 0
    with pytest.raises(W.WldError):
        ctx.run_wait()  # nothing in flight


def test_contexts_on_one_stream(W):
    # wld_set_stream: three contexts on the first one's stream, runs enqueued
    # back to back (no event between them; wld_run_after a no-op), each
    # context's rows bit-identical to the oracle's in lib.rs's order; back on
    # its own stream afterwards; refused during a run.
    L, N = 600, 300
    buf = synth(L, N, 91)
    w = np.random.default_rng(9).random(N).astype(np.float32) + 0.05
    cs = [W.Context(0) for _ in range(3)]
    for c in cs:
        c.load(buf, w)
    for c in cs[1:]:
        c.set_stream(cs[0])
        assert c.stream_ptr() == cs[0].stream_ptr()
    thrs = [0.0, 0.02, 0.3, 0.02, 0.0, 0.3]
    refs = {t: O.all_pairs(buf, w, np.float32(t)) for t in set(thrs)}
    pend = []
    for i, t in enumerate(thrs):
        c = cs[i % 3]
        if pend and pend[0][0] is c:
            pc, pt = pend.pop(0)
            assert pc.run_wait() == len(refs[pt]["site_a"])
            _bit_equal_rows(pc.rows(), refs[pt])
        if pend:
            c.run_after(pend[-1][0])
        c.run_chunks_async(t, 0, 0)
        pend.append((c, t))
        if i == 2:
            with pytest.raises(W.WldError):
                c.set_stream(None)  # during its run
    for pc, pt in pend:
        assert pc.run_wait() == len(refs[pt]["site_a"])
        _bit_equal_rows(pc.rows(), refs[pt])
    cs[1].set_stream(None)
    assert cs[1].stream_ptr() not in (0, cs[0].stream_ptr())
    assert cs[1].run(0.02) == len(refs[0.02]["site_a"])
    _bit_equal_rows(cs[1].rows(), refs[0.02])
    # the owner closed while cs[2] still runs on its stream: cs[2] gets its
    # own stream back first and keeps working
    cs[2].run_chunks_async(0.0, 0, 0)
    with pytest.raises(W.WldError):
        cs[0].close()  # cs[2] has a run in flight on cs[0]'s stream: refused, nothing destroyed
    assert cs[2].run_wait() == len(refs[0.0]["site_a"])
    cs[0].close()
    assert cs[2].stream_ptr() not in (0,)
    assert cs[2].run(0.3) == len(refs[0.3]["site_a"])
    _bit_equal_rows(cs[2].rows(), refs[0.3])


def _bit_equal_rows(store, ref):
    assert np.array_equal(store.site_a.astype(np.uint64), ref["site_a"])
    assert np.array_equal(store.site_b.astype(np.uint64), ref["site_b"])
    for f in ("d", "d_prime", "r2"):
        g, r = getattr(store, f), np.asarray(ref[f], dtype=np.float32)
        assert np.array_equal(g.view(np.uint32), r.view(np.uint32)) or \
            np.all((g.view(np.uint32) == r.view(np.uint32)) | (np.isnan(g) & np.isnan(r))), f


def test_shard_step_world1_rccl(W, ctxs):
    # ShardStep (the bench's N>1 step) through a real world-1 RCCL group: the
    # count all_gather ordered on the library's stream, then the rows.
    import torch
    import torch.distributed as dist
    from weightedld_amd import dist as wdist

    ctx = _ctx(ctxs, "mfma")
    L, N = 700, 256
    buf = synth(L, N, 78)
    w = np.random.default_rng(4).random(N).astype(np.float32) + 0.1
    ctx.load(buf, w)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        step = wdist.ShardStep(ctx, 0, 1, dev)
        for thr in (0.0, 0.02, 2.0):
            ref = O.all_pairs(buf, w, thr)
            for _ in range(2):
                n, rows = step(thr, 0, 0)
                got = wdist.unpack_rows(rows)
                assert n == rows.shape[1]
                assert list(zip(got["site_a"].tolist(), got["site_b"].tolist())) == \
                    list(zip(ref["site_a"].tolist(), ref["site_b"].tolist()))
                assert np.abs(got["r2"].astype(np.float64) - ref["r2"]).max(initial=0.0) < 1e-5
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("serialize,depth", [(False, 2), (True, 2), ("pair", 2), ("pair", 3), (False, 3)])
def test_pipelined_shard_step_world1_rccl(W, serialize, depth):
    # PipelinedShardStep (the bench's N>1 timed loop): two contexts on the same
    # inputs, step i's kernel queued behind step i-1's on the device while
    # step i-1 completes.  Every step's rows equal the oracle's, in order,
    # across threshold changes, steps with and without rows, and a drain.
    import torch
    import torch.distributed as dist
    from weightedld_amd import dist as wdist

    L, N = 700, 256
    buf = synth(L, N, 79)
    w = np.random.default_rng(8).random(N).astype(np.float32) + 0.1
    ctxs2 = [W.Context(0, W.KERNEL_MFMA) for _ in range(depth)]
    for c in ctxs2:
        c.load(buf, w)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = "29562"
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        pipe = wdist.PipelinedShardStep(ctxs2, 0, 1, dev, serialize_kernels=serialize)
        thrs = [0.0, 0.02, 2.0, 0.02, 0.0, 2.0, 2.0, 0.01]
        refs = {t: O.all_pairs(buf, w, t) for t in set(thrs)}
        results = []
        for i, t in enumerate(thrs):
            r = pipe.submit(t, 0, 0)
            assert (r is None) == (i < depth - 1)
            if r is not None:
                results.append(r)
        results += pipe.drain_all()
        assert pipe.drain() is None
        assert len(results) == len(thrs)
        for t, (n, rows) in zip(thrs, results):
            ref = refs[t]
            got = wdist.unpack_rows(rows)
            assert n == rows.shape[1] == len(ref["site_a"])
            assert list(zip(got["site_a"].tolist(), got["site_b"].tolist())) == \
                list(zip(ref["site_a"].tolist(), ref["site_b"].tolist()))
            assert np.abs(got["r2"].astype(np.float64) - ref["r2"]).max(initial=0.0) < 1e-5
    finally:
        dist.destroy_process_group()
        for c in ctxs2:
            c.close()


def test_run_host_batches_concatenate(W, ctxs):
    # wld_run_host / wld_all_weighted_ld_pairs split the chunk sequence into
    # batches (<= 2^31 pairs; forced small here) and append their rows: the
    # result equals one run, in reference order, with per-batch progress.
    ctx = _ctx(ctxs, "mfma")
    L, N = 1100, 200
    buf = synth(L, N, 90)
    w = np.random.default_rng(6).random(N).astype(np.float32) + 0.1
    ref = O.all_pairs(buf, w, 0.01)
    ctx.load(buf, w)
    whole = ctx.run_host(0.01)
    ctx.set_option("host_batch_pairs", 70000)  # about one chunk per batch
    seen = []
    got = ctx.run_host(0.01, seen.append)
    # one call per chunk (lib.rs:670-674) across batches, the counter before each chunk's add
    assert len(seen) == ctx.chunks(L) and seen == sorted(seen) and seen[0] == 0 and seen[-1] < L * (L - 1) // 2
    for f in ("site_a", "site_b", "d", "d_prime", "r2"):
        assert np.array_equal(getattr(got, f).view(np.uint32), getattr(whole, f).view(np.uint32)), f
    compare_rows(got, ref, 0.01, buf=buf, w=w)
    store = W.all_weighted_ld_pairs(W.SiteSet.from_buffer(buf), w, 0.01, ctx=ctx)
    assert np.array_equal(store.site_a, got.site_a) and np.array_equal(store.r2.view(np.uint32),
                                                                       got.r2.view(np.uint32))
    ctx.set_option("host_batch_pairs", 1 << 31)


@pytest.mark.parametrize("devices", [None, [0, 0], [0, 0, 0]])
def test_progress_once_per_chunk_config2(W, devices):
    """lib.rs reports progress once per 256x256 chunk (lib.rs:670-674, after
    the initial 0 of :584): at BASELINE config 2 (2000 sites: 36 chunks) the
    drop-in calls back 37 times, on the calling thread, with the running
    count of pairs in the chunks finished before each one — values that never
    decrease and step by whole chunks — single-device and as a device group."""
    import threading
    sys_path_bench()
    from bench import synth as bench_synth
    from bench import chunk_pairs
    L, N = 2000, 500
    buf = bench_synth(L, N)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    ctx = W.Context(0, devices=devices) if devices else W.Context(0)
    seen, threads = [], set()

    def cb(n):
        seen.append(n)
        threads.add(threading.get_ident())
    store = W.all_weighted_ld_pairs(W.SiteSet.from_buffer(buf), w, 0.0, progress_report=cb, ctx=ctx)
    n_chunks = ctx.chunks(L)
    assert n_chunks == 36
    assert len(seen) == 1 + n_chunks, len(seen)
    assert seen[0] == 0 and seen[1] == 0 and seen == sorted(seen)
    assert threads == {threading.get_ident()}
    steps = sorted(np.diff(seen[1:]).tolist() + [L * (L - 1) // 2 - seen[-1]])
    assert steps == sorted(chunk_pairs(L, i) for i in range(n_chunks))
    assert ctx.stats()["progress_filled"] == 0  # every chunk's report came from the kernels' log
    assert len(store) > 1_990_000



@pytest.mark.parametrize("thr,screen,fp6", [(0.05, 1, 0), (0.002, 4, 0), (0.05, 1, 2)],
                         ids=["screen_items", "candidate_pairs", "fp6_screen"])
def test_progress_once_per_chunk_screened(W, thr, screen, fp6):
    """Per-chunk progress through the screened paths on linkage-block data:
    at 0.05 the i8 (or, forced, the fp6) screen and the f32 candidate launch
    over 16-row-block items (a chunk finishes when the screen's rejected row
    blocks and every item's row block are done), at 0.002 the exact candidate
    pairs (a tile is done after ref_compact).  One callback per chunk, values
    in lib.rs's fetch_add sequence, none made up by the host; the rows equal
    the oracle's bit for bit."""
    sys_path_bench()
    from bench import chunk_pairs, ld_blocks
    L, N = 3000, 600
    buf = ld_blocks(L, N)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    ctx = W.Context(0)
    ctx.set_option("screen", screen)
    ctx.set_option("screen_fp6", fp6)
    seen = []
    store = W.all_weighted_ld_pairs(W.SiteSet.from_buffer(buf), w, thr, progress_report=seen.append, ctx=ctx)
    st = ctx.stats()
    assert st["screened"] == screen and st["candidate_tiles"] > 0, st
    assert st["screen_fp6"] == (1 if fp6 else 0), st
    assert st["progress_filled"] == 0, st
    n_chunks = ctx.chunks(L)
    assert len(seen) == 1 + n_chunks and seen[0] == 0 and seen == sorted(seen)
    steps = sorted(np.diff(seen[1:]).tolist() + [L * (L - 1) // 2 - seen[-1]])
    assert steps == sorted(chunk_pairs(L, i) for i in range(n_chunks))
    ref = O.all_pairs(buf, w, np.float32(thr))
    assert len(store) == len(ref["r2"]) > 0
    assert np.array_equal(store.site_a.astype(np.uint64), ref["site_a"])
    assert np.array_equal(store.r2.view(np.uint32), ref["r2"].view(np.uint32))
    ctx.close()


# ------------------------------------------------------------------ CLI progress bars (main.rs:89-116, 170-190)
def _write_c2_fasta(path):
    sys_path_bench()
    from bench import synth as bench_synth
    codes = bench_synth(2000, 500)  # BASELINE config 2: 500 sequences x 2000 sites, all kept
    lut = np.frombuffer(b"ACGT-N", dtype=np.uint8)
    with open(path, "wb") as f:
        for k in range(codes.shape[1]):
            f.write(b">s%d\n" % k + lut[codes[:, k]].tobytes() + b"\n")


@pytest.mark.parametrize("prepass", [False, True], ids=["host_prepass", "gpu_prepass"])
def test_cli_progress_bars(tmp_path, prepass):
    """The CLI feeds the LD pass's progress_report closure (main.rs:184-188) to
    a progress bar: at BASELINE config 2 (36 chunks) the closure is called 37
    times (progress(0), then one per chunk; logged at debug level).  The bars
    (LD pass and TSV write, indicatif's template) are drawn only when info is
    enabled AND stderr is a terminal (here forced with the CLI's test hook
    WLD_FORCE_PROGRESS_BAR: the GPU box has no pseudo-terminals); the TSV is
    byte-identical either way, and with stderr on a pipe the log lines carry
    no bar."""
    fa = tmp_path / "c2.fasta"
    _write_c2_fasta(fa)
    extra = ["--gpu-prepass"] if prepass else []
    env = dict(os.environ)

    def cmd(out):
        return [CLI, "--fasta-input", str(fa), "--pair-output", str(out), "--r2-threshold", "0.0"] + extra

    # debug level, stderr on a pipe: the closure's call count, no bar
    r = subprocess.run(cmd(tmp_path / "a.tsv"), capture_output=True, text=True, timeout=120,
                       env=dict(env, RUST_LOG="debug"))
    assert r.returncode == 0, r.stderr
    m = re.search(r"progress: (\d+) progress_report calls, last (\d+) pairs", r.stderr)
    assert m, r.stderr[-2000:]
    assert int(m.group(1)) == 37
    assert 0 < int(m.group(2)) < 2000 * 1999 // 2  # the last value: every pair but the last chunk's
    assert "\x1b[2K" not in r.stderr and "pairs computed at" in r.stderr
    # info level on a terminal: bar frames on stderr, same TSV, and the same
    # log lines once the frames are taken out
    # (bytes, decoded by hand: text mode would turn every "\r" into a newline)
    r2 = subprocess.run(cmd(tmp_path / "b.tsv"), capture_output=True, timeout=120,
                        env=dict(env, RUST_LOG="info", WLD_FORCE_PROGRESS_BAR="1"))
    r2.stderr = r2.stderr.decode("utf-8")
    assert r2.returncode == 0, r2.stderr[-2000:]
    assert "\x1b[2K" in r2.stderr and re.search(r"\] \d+% \(\d+/s \d\d:\d\d:\d\d\)", r2.stderr), r2.stderr[-2000:]
    assert (tmp_path / "b.tsv").read_bytes() == (tmp_path / "a.tsv").read_bytes()
    plain = subprocess.run(cmd(tmp_path / "d.tsv"), capture_output=True, text=True, timeout=120,
                           env=dict(env, RUST_LOG="info"))
    # a frame is "\r\x1b[2K\x1b[32m<spinner>...", up to the next frame or the clear "\r\x1b[2K"
    unbar = lambda t: re.sub(r"\r\x1b\[2K", "", re.sub(r"\r\x1b\[2K\x1b\[32m[^\r\n]*", "", t))  # noqa: E731
    strip = lambda t: [re.sub(r"\[\S+Z ", "[", ln) for ln in unbar(t).splitlines()]  # noqa: E731
    assert "\x1b[2K" not in plain.stderr
    keep = lambda t: [ln for ln in strip(t) if not re.search(r"computed at| in \d|Writing output", ln)]  # noqa: E731
    assert keep(r2.stderr) == keep(plain.stderr) and len(keep(plain.stderr)) >= 3, (keep(r2.stderr), keep(plain.stderr))
    # warn level: no bar (log_enabled!(Level::Info) is false)
    r3 = subprocess.run(cmd(tmp_path / "c.tsv"), capture_output=True, text=True, timeout=120,
                        env=dict(env, RUST_LOG="warn", WLD_FORCE_PROGRESS_BAR="1"))
    assert r3.returncode == 0 and "\x1b[2K" not in r3.stderr and "%" not in r3.stderr, r3.stderr[-2000:]
    assert (tmp_path / "c.tsv").read_bytes() == (tmp_path / "a.tsv").read_bytes()
