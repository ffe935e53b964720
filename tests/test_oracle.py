"""Pin the CPU oracle (oracle/wld_oracle.c) before trusting it as the checker.

1. lib.rs unit-test known answers (lib.rs:686-802), committed as data in
   tests/golden/librs_known_answers.json.
2. Golden vectors produced by running the Python reference (WeightedLD.py) under
   oracle/gen_golden.py, on the sub-domain where Python and lib.rs semantics
   coincide: no Unknown symbols, constant distinct
   symbol count per site, Python's skip rule applied on top.
"""
import math
import os

import numpy as np
import pytest

import _oracle as O
from conftest import FIXTURES, SYNTH

TOL = 1e-5  # north_star: D, D' and r2 within 1e-5 (f32)


# ---------------------------------------------------------------- known answers
def test_histogram_known_answer(librs_ka):
    ka = librs_ka["histogram"]
    h = O.histogram(O.symbols(ka["symbols"]))
    assert list(h) == ka["expect"]


def test_major_minor_known_answers(librs_ka):
    for c in librs_ka["major_minor"]["cases"]:
        assert O.major_minor(c["hist"]) == (c["major"], c["minor"])


def test_major_minor_none():
    assert O.major_minor([0, 0, 0, 0, 0, 7]) == (None, None)
    assert O.major_minor([5, 0, 0, 0, 0, 3]) == (0, None)
    # ties keep the earlier symbol (strict '>' at lib.rs:131,134)
    assert O.major_minor([4, 4, 0, 0, 0, 0]) == (0, 1)
    assert O.major_minor([0, 0, 3, 3, 3, 0]) == (2, 3)


def _siteset_from_strs(seqs):
    return np.stack([O.symbols(s) for s in seqs], axis=1)  # [site, seq]


def test_henikoff_known_answers(librs_ka):
    for c in librs_ka["henikoff"]["cases"]:
        w = O.henikoff_weights(_siteset_from_strs(c["seqs"]))
        exp = np.array(c["expect"], dtype=np.float32)
        if c["tol"] == "ulps":
            assert np.all(np.abs(w.view(np.int32) - exp.view(np.int32)) <= 4), (w, exp)
        else:
            assert np.allclose(w, exp, atol=c["tol"], rtol=0), (w, exp)


def test_ld_pair_known_answers(librs_ka):
    for c in librs_ka["ld_pair"]["cases"]:
        r = O.single_pair(O.symbols(c["a"]), O.symbols(c["b"]), c["w"])
        assert r is not None
        d, dp, r2 = r
        assert abs(d - c["d"]) <= c["tol"], (c["ref"], r)
        assert abs(dp - c["d_prime"]) <= c["tol"], (c["ref"], r)
        assert abs(r2 - c["r2"]) <= c["tol"], (c["ref"], r)


def test_ld_pair_none_when_monomorphic():
    a = O.symbols("AAAAAAAAA")
    b = O.symbols("ACACACACA")
    assert O.single_pair(a, b, np.ones(9)) is None


def test_triu_index_covers_upper_triangle_once():
    for L in (1, 255, 256, 257, 2000, 20000, 50000):
        n = L // 256 + (L % 256 > 0)
        seen = set()
        prev_row = None
        for i in range(n * (n + 1) // 2):
            r, c = O.triu_index(n, i)
            assert 0 <= r <= c < n
            seen.add((r, c))
            if prev_row is not None:
                assert r <= prev_row  # chunk rows descend (lib.rs:628)
            prev_row = r
        assert len(seen) == n * (n + 1) // 2


# ---------------------------------------------------------------- FASTA reader
def test_read_fasta_trailing_unknown_site():
    buf = O.read_fasta(os.path.join(FIXTURES, "example.fasta"))
    # 4 symbols + the '\n' kept by read_line → 5 sites, last one Unknown (lib.rs:289-297)
    assert buf.shape == (5, 10)
    assert np.all(buf[4] == 5)


def test_read_fasta_panics_without_final_newline():
    # t1 has no trailing newline, so its last sequence is one symbol short and
    # SiteSet::from_multiseq panics (lib.rs:180-182).
    with pytest.raises(ValueError):
        O.read_fasta(os.path.join(FIXTURES, "t1_henikoff_paper.fasta"))


# ---------------------------------------------------------------- Python goldens
def _oracle_dense_lookup(buf, w):
    d, dp, r2, valid = O.all_pairs_dense(buf, w)
    return d, dp, r2, valid


@pytest.mark.parametrize("name", ["synth_n200_l24.fasta", "synth_n500_l40.fasta", "synth_n2000_l30.fasta"])
def test_synthetic_vs_python_reference(python_ref, name):
    g = python_ref[name]
    buf = O.read_fasta(os.path.join(SYNTH, name))[:-1]  # drop the trailing '\n' Unknown site
    assert buf.shape == (g["n_sites"], g["n_seqs"])
    mask = O.site_mask(buf)
    assert list(mask) == g["var_sites_ld"]
    sub = buf[mask]
    site_map = np.nonzero(mask)[0]
    w = O.henikoff_weights(sub)
    assert np.allclose(w, np.array(g["weights"]), rtol=2e-6, atol=0)
    for weights, key in ((w, "pairs_weighted"), (np.ones_like(w), "pairs_unweighted")):
        d, dp, r2, valid = _oracle_dense_lookup(sub, weights)
        rows = g[key]
        L = sub.shape[0]
        assert len(rows) == L * (L - 1) // 2  # no Python skips on this domain
        idx = {int(s): i for i, s in enumerate(site_map)}
        worst = 0.0
        for a, b, D, Dp, R2 in rows:
            i, j = idx[a], idx[b]
            assert valid[i, j]
            for mine, ref in ((d[i, j], D), (dp[i, j], Dp), (r2[i, j], R2)):
                worst = max(worst, abs(float(mine) - ref))
        assert worst <= TOL, worst


def _vcf_buffer(g):
    return np.array([[int(ch) for ch in col] for col in g["alignment_T"]], dtype=np.uint8)


def test_vcf_weighted_vs_python_reference(python_ref):
    # BASELINE config 3.  handle_vcf (WeightedLD.py:311-379) gives 5 sites x 5008
    # haplotypes with allele digits as symbol codes; the lib.rs pair math with
    # lib.rs Henikoff weights reproduces Python's 10 unrounded rows.
    g = python_ref["t7_1000genome.vcf"]
    buf = _vcf_buffer(g)
    assert buf.shape == (5, 5008)
    assert round(float(np.mean(g["weights"])), 3) == 0.002  # dead test.py:152-159
    w = O.henikoff_weights(buf)
    d, dp, r2, valid = O.all_pairs_dense(buf, w)
    sm = g["site_map"]
    assert len(g["pairs_weighted"]) == 10
    for a, b, D, Dp, R2 in g["pairs_weighted"]:
        i, j = sm.index(a), sm.index(b)
        assert valid[i, j]
        assert abs(d[i, j] - D) <= TOL
        assert abs(dp[i, j] - Dp) <= TOL
        assert abs(r2[i, j] - R2) <= TOL


def test_vcf_unweighted_matches_python_skip_rule(python_ref):
    # Python prints nothing unweighted because every pair trips the
    # round(PA,1)==1.0 skip (WeightedLD.py:234-237): the rare allele makes PA > 0.95.
    g = python_ref["t7_1000genome.vcf"]
    assert g["pairs_unweighted"] == []
    buf = _vcf_buffer(g)
    for s in range(buf.shape[0]):
        h = O.histogram(buf[s])
        maj, mnr = O.major_minor(h)
        assert h[maj] / (h[maj] + h[mnr]) >= 0.95


def test_fixture_t2_matches_python(python_ref):
    # t2 lies in the parity domain: one LD pair (1,2)
    g = python_ref["t2_henikoff_complex1.fasta"]
    buf = O.read_fasta(os.path.join(FIXTURES, "t2_henikoff_complex1.fasta"))[:-1]
    mask = O.site_mask(buf)
    assert list(mask) == g["var_sites_ld"]
    sub = buf[mask]
    w = O.henikoff_weights(sub)
    res = O.all_pairs(sub, w, float("-inf"), site_map=np.nonzero(mask)[0])
    (a, b, D, Dp, R2), = g["pairs_weighted"]
    assert (int(res["site_a"][0]), int(res["site_b"][0])) == (a, b)
    assert abs(res["d"][0] - D) <= TOL and abs(res["d_prime"][0] - Dp) <= TOL and abs(res["r2"][0] - R2) <= TOL


def test_example_fasta_librs_semantics():
    # example.fasta is OUTSIDE the Python parity domain (one 'y', mixed distinct
    # counts): SURVEY.md App. D gives the lib.rs-derived CLI row 0 1 0.107 0.345 0.237.
    buf = O.read_fasta(os.path.join(FIXTURES, "example.fasta"))
    mask = O.site_mask(buf)
    assert list(np.nonzero(mask)[0]) == [0, 1]
    sub = buf[mask]
    w = O.henikoff_weights(sub)
    assert ["%.3f" % x for x in w] == ["1.000", "0.300", "0.300", "0.300", "0.700"] + ["0.200"] * 5
    res = O.all_pairs(sub, w, 0.1, site_map=np.nonzero(mask)[0])
    assert res["site_a"].tolist() == [0] and res["site_b"].tolist() == [1]
    assert "%.3f\t%.3f\t%.3f" % (res["d"][0], res["d_prime"][0], res["r2"][0]) == "0.107\t0.345\t0.237"
    res_u = O.all_pairs(sub, np.ones_like(w), 0.1, site_map=np.nonzero(mask)[0])
    assert res_u["site_a"].size == 0  # r2 = 0.0625 <= 0.1


def test_all_pairs_order_and_threshold():
    rng = np.random.default_rng(5)
    L, N = 600, 40
    buf = rng.integers(0, 5, size=(L, N)).astype(np.uint8)
    w = rng.random(N).astype(np.float32)
    res = O.all_pairs(buf, w, 0.0, n_threads=4)
    assert res["pairs"] == L * (L - 1) // 2
    # rows come chunk by chunk in triu order, a then b ascending within a chunk
    n = (L + 255) // 256
    order = []
    for i in range(n * (n + 1) // 2):
        ca, cb = O.triu_index(n, i)
        order.append((ca, cb))
    rank = {c: k for k, c in enumerate(order)}
    key = [(rank[(int(a) // 256, int(b) // 256)], int(a), int(b)) for a, b in zip(res["site_a"], res["site_b"])]
    assert key == sorted(key)
    assert np.all(res["r2"] > 0.0)
    d, dp, r2, valid = O.all_pairs_dense(buf, w)
    iu = np.triu_indices(L, 1)
    passing = np.sum((valid[iu] == 1) & (r2[iu] > 0.0))
    assert passing == res["site_a"].size
