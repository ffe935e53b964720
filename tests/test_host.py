"""CPU tests of the product library's host side and C ABI (no GPU compute).

* libweightedld.so loads and exports every function include/weightedld.h declares.
* The C++ host pre-pass (FASTA reader, site filter, Henikoff weights, VCF
  reader) agrees bit-for-bit with the oracle restatement and the Python
  reference goldens.
* Shard planning covers the chunk rows exactly once with balanced pair counts.
* The device entry points fail loudly (WLD_E_NODEV) where there is no GPU.
"""
import os
import re
import subprocess

import numpy as np
import pytest

import _oracle as O
from conftest import CLI, FIXTURES, REPO, SYNTH

import weightedld_amd as W
from weightedld_amd import _lib

HEADER = os.path.join(REPO, "include", "weightedld.h")


def _gpu_present():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def test_library_exports_every_header_symbol():
    src = open(HEADER).read()
    declared = set(re.findall(r"\b(wld_[a-z0-9_]+)\s*\(", src))
    declared -= {"wld_progress_fn"}
    assert declared, "no declarations parsed"
    lib = W.lib()
    missing = [s for s in sorted(declared) if not hasattr(lib, s)]
    assert not missing, missing
    # and the ctypes signature table covers them all
    assert declared <= set(_lib.SIGNATURES), sorted(declared - set(_lib.SIGNATURES))
    nm = subprocess.run(["nm", "-D", "--defined-only", W.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (wld_[a-z0-9_]+)", nm))
    assert declared <= exported, sorted(declared - exported)


def test_version_and_status_strings():
    assert b"gfx950" in W.lib().wld_version()
    assert W.lib().wld_status_string(-4) == b"no gfx950 device"


ALL_FASTA = ["example.fasta", "t2_henikoff_complex1.fasta", "t3_henikoff_complex2.fasta",
             "t4_weights1_ld0.fasta", "t5_weights1_ld0.25.fasta", "t6_varsites_hk_ld.fasta"]


@pytest.mark.parametrize("name", ALL_FASTA + ["synthetic/synth_n500_l40.fasta", "synthetic/synth_n2000_l30.fasta"])
def test_read_fasta_matches_oracle(name):
    path = os.path.join(FIXTURES if "/" not in name else os.path.dirname(SYNTH), name)
    ss = W.read_fasta(path)
    ref = O.read_fasta(path)
    assert (ss.n_sites(), ss.n_seqs()) == ref.shape
    assert np.array_equal(ss.buffer, ref)
    for i in range(ref.shape[0]):
        assert np.array_equal(ss.site_histogram(i).data, O.histogram(ref[i]))


@pytest.mark.parametrize("n_seqs,n_sites", [(1, 1), (63, 65), (130, 257), (200, 1000)])
def test_read_fasta_blocked_transpose_vs_oracle(tmp_path, n_seqs, n_sites):
    # ragged 64x64 blocks, every byte class (upper/lower ACGT, '-', others, a
    # header-like '>' inside no line), histograms fused into the transpose
    rng = np.random.default_rng(n_seqs * 7 + n_sites)
    alphabet = np.frombuffer(b"ACGTacgt-NnXx*.?", dtype=np.uint8)
    lines = []
    for q in range(n_seqs):
        lines.append(b">seq%d description\n" % q)
        lines.append(alphabet[rng.integers(0, len(alphabet), n_sites)].tobytes() + b"\n")
    p = tmp_path / "r.fasta"
    p.write_bytes(b"".join(lines))
    ss = W.read_fasta(str(p))
    ref = O.read_fasta(str(p))
    assert (ss.n_sites(), ss.n_seqs()) == ref.shape
    assert np.array_equal(ss.buffer, ref)
    for i in range(0, ref.shape[0], max(1, ref.shape[0] // 50)):
        assert np.array_equal(ss.site_histogram(i).data, O.histogram(ref[i]))


def test_read_fasta_panic_cases(tmp_path):
    with pytest.raises(W.WldError) as e:
        W.read_fasta(os.path.join(FIXTURES, "t1_henikoff_paper.fasta"))
    assert e.value.name == "WLD_E_FORMAT"
    # the message reads the lengths before the half-built set is freed (a
    # use-after-free here once printed garbage and corrupted the heap)
    assert "sequence 4 has 7, sequence 0 has 8" in str(e.value)
    for _ in range(3):
        r = subprocess.run([CLI, "--fasta-input", os.path.join(FIXTURES, "t1_henikoff_paper.fasta"), "--pair-output",
                            str(tmp_path / "p.tsv")], capture_output=True, text=True, timeout=60)
        assert r.returncode == 101 and "sequence 0 has 8;" in r.stderr, r.stderr
    p = tmp_path / "empty.fasta"
    p.write_text(">only a header\n")
    with pytest.raises(W.WldError):
        W.read_fasta(str(p))
    with pytest.raises(W.WldError) as e:
        W.read_fasta(str(tmp_path / "missing.fasta"))
    assert e.value.name == "WLD_E_IO"


def test_read_fasta_crlf_and_utf8(tmp_path):
    p = tmp_path / "crlf.fasta"
    p.write_bytes(b">a\r\nACGT\r\n>b\r\nAC-T\r\n")
    ss = W.read_fasta(str(p))
    assert ss.n_sites() == 6  # 4 symbols + '\r' + '\n', both Unknown
    assert ss.buffer[:, 1].tolist() == [0, 1, 4, 3, 5, 5]
    q = tmp_path / "utf8.fasta"
    q.write_bytes(">a\nACéT\n>b\nACGT\n".encode())
    ss = W.read_fasta(str(q))  # 'é' is one char (one Unknown site) for Rust's chars()
    assert ss.n_sites() == 5 and ss.buffer[2, 0] == 5


def test_major_minor_known_answers(librs_ka):
    for c in librs_ka["major_minor"]["cases"]:
        mj, mn = W.SymbolHistogram(c["hist"]).major_minor_symbols()
        assert (int(mj), int(mn)) == (c["major"], c["minor"])
    h = W.SymbolHistogram.from_slice(W.api.symbols_from_str(librs_ka["histogram"]["symbols"]))
    assert h.data.tolist() == librs_ka["histogram"]["expect"]


def test_henikoff_known_answers(librs_ka):
    for c in librs_ka["henikoff"]["cases"]:
        w = W.henikoff_weights(W.SiteSet.from_strs(c["seqs"]))
        exp = np.array(c["expect"], dtype=np.float32)
        tol = 1e-6 if c["tol"] == "ulps" else c["tol"]
        assert np.allclose(w, exp, atol=tol, rtol=0), (w, exp)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_filter_and_henikoff_bitexact_vs_oracle(seed):
    rng = np.random.default_rng(seed)
    L, N = 300, 257
    buf = rng.choice(6, size=(L, N), p=[0.35, 0.25, 0.1, 0.1, 0.12, 0.08]).astype(np.uint8)
    buf[5] = 0  # monomorphic site
    buf[6, :] = 5  # all Unknown
    ss = W.SiteSet.from_buffer(buf)
    for args in ((0.8, 0.02, 0.5), (0.5, 0.1, 0.45), (0.0, 0.0, 1.0)):
        f = ss.filter_sites_of_interest(*args)
        mask = O.site_mask(buf, *args)
        assert f.site_map.tolist() == list(np.nonzero(mask)[0])
        assert np.array_equal(f.buffer, buf[mask])
        if f.n_sites():
            w = W.henikoff_weights(f)
            wo = O.henikoff_weights(buf[mask])
            assert np.array_equal(w.view(np.uint32), wo.view(np.uint32))
    w = W.henikoff_weights(ss)
    wo = O.henikoff_weights(buf)
    assert np.array_equal(np.isnan(w), np.isnan(wo))
    assert np.array_equal(w[~np.isnan(w)].view(np.uint32), wo[~np.isnan(wo)].view(np.uint32))


def test_is_site_of_interest_matches_oracle():
    rng = np.random.default_rng(7)
    for _ in range(200):
        n = int(rng.integers(1, 60))
        site = rng.integers(0, 6, size=n).astype(np.uint8)
        k = int(rng.integers(0, n + 1))
        lo, hi = sorted(rng.random(2))
        assert W.is_site_of_interest(site, k, lo, hi) == bool(
            O.lib().wldo_is_site_of_interest(site.ctypes.data_as(O.ctypes.POINTER(O.ctypes.c_uint8)), n, k, lo, hi))


def test_zero_sites_weights_are_nan():
    ss = W.SiteSet.from_buffer(np.zeros((0, 4), dtype=np.uint8))
    assert np.all(np.isnan(W.henikoff_weights(ss)))  # 0/0


def test_vcf_reader_matches_python_handle_vcf(python_ref):
    g = python_ref["t7_1000genome.vcf"]
    ss = W.read_vcf(os.path.join(FIXTURES, "t7_1000genome.vcf"))
    assert (ss.n_sites(), ss.n_seqs()) == (g["n_sites"], g["n_seqs"])
    assert ss.site_map.tolist() == g["site_map"]
    exp = np.array([[int(c) for c in col] for col in g["alignment_T"]], dtype=np.uint8)
    assert np.array_equal(ss.buffer, exp)


def test_vcf_reader_errors(tmp_path):
    p = tmp_path / "nohdr.vcf"
    p.write_text("##fileformat=VCFv4.2\n1\t2\t3\n")
    with pytest.raises(W.WldError) as e:
        W.read_vcf(str(p))
    assert e.value.name == "WLD_E_FORMAT"
    q = tmp_path / "small.vcf"
    q.write_text("#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tA\n1\t5\t.\tA\tT\t1\tP\t.\tGT\t0|1\n")
    with pytest.raises(W.WldError):
        W.read_vcf(str(q))


@pytest.mark.parametrize("L", [0, 1, 255, 256, 257, 2000, 20000, 50000])
@pytest.mark.parametrize("G", [1, 2, 3, 4, 8])
def test_shard_partition(L, G):
    n = W.Context.chunk_rows(L)
    assert n == (L + 255) // 256
    spans = [W.Context.shard_chunk_rows(L, G, g) for g in range(G)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (b0, e0), (b1, e1) in zip(spans, spans[1:]):
        assert e0 == b1 and b0 <= e0
    if L >= 20000:
        # balanced to within one chunk row's worth of pairs
        def pairs(rb, re_):
            a0, a1 = min(L, rb * 256), min(L, re_ * 256)
            return sum(L - 1 - a for a in range(a0, a1))
        tot = L * (L - 1) // 2
        for b, e in spans:
            assert abs(pairs(b, e) - tot / G) <= 256 * L


@pytest.mark.parametrize("L", [0, 1, 255, 256, 257, 700, 2000, 20000, 50000])
@pytest.mark.parametrize("G", [1, 2, 3, 4, 8])
def test_shard_chunks_partition(L, G):
    """wld_shard_chunks: contiguous linear chunk ranges, shard 0 LAST, covering
    all n(n+1)/2 chunks, pair counts (wld_pairs_in_chunks) summing to L(L-1)/2
    and each within one chunk (256^2 pairs) of the even share."""
    n = W.Context.chunk_rows(L)
    m = W.Context.chunks(L)
    assert m == n * (n + 1) // 2
    spans = [W.Context.shard_chunks(L, G, g) for g in range(G)]
    assert spans[-1][0] == 0 and spans[0][1] == m
    for (b0, e0), (b1, e1) in zip(spans, spans[1:]):
        assert b0 == e1 and b0 <= e0  # shard g+1 ends where shard g begins
    pairs = [W.Context.pairs_in_chunks(L, b, e) for b, e in spans]
    assert sum(pairs) == L * (L - 1) // 2
    for p in pairs:
        assert abs(p - L * (L - 1) / 2 / G) <= 256 * 256
    # a whole-row range counts the same pairs as the row formula
    if n:
        lin = lambda r, c: (n - 1 - r) * (n - r) // 2 + (c - r)  # noqa: E731
        rb, re_ = 0, max(1, n // 2)
        a0, a1 = 0, min(L, re_ * 256)
        assert W.Context.pairs_in_chunks(L, lin(re_ - 1, re_ - 1), lin(rb, rb) + n - rb) == \
            sum(L - 1 - a for a in range(a0, a1))


@pytest.mark.skipif(_gpu_present(), reason="checks the no-GPU error path")
def test_device_entry_points_fail_loudly_without_gpu():
    with pytest.raises(W.WldError) as e:
        W.Context(0)
    assert e.value.name == "WLD_E_NODEV"


def test_cli_help_and_arg_errors(tmp_path):
    r = subprocess.run([CLI, "--help"], capture_output=True, text=True)
    assert r.returncode == 0 and "--fasta-input" in r.stdout and "--r2-threshold" in r.stdout
    r = subprocess.run([CLI, "--pair-output", str(tmp_path / "x.tsv")], capture_output=True, text=True)
    assert r.returncode == 1 and "--fasta-input" in r.stderr
    r = subprocess.run([CLI, "--fasta-input", "x", "--pair-output", "y", "--bogus"], capture_output=True, text=True)
    assert r.returncode == 1


@pytest.mark.parametrize("rust_log", [None, "error"])
def test_cli_exact_sums_warns(tmp_path, rust_log):
    # --exact-sums is this build's addition, not a reference flag (main.rs:14-68):
    # its TSV is not lib.rs's, so the CLI says so on stderr at any log level,
    # before any GPU step (checkable here, without a device)
    env = dict(os.environ)
    if rust_log:
        env["RUST_LOG"] = rust_log
    r = subprocess.run([CLI, "--fasta-input", os.path.join(FIXTURES, "example.fasta"), "--pair-output",
                        str(tmp_path / "p.tsv"), "--exact-sums"], capture_output=True, text=True, env=env)
    assert "WARN" in r.stderr and "--exact-sums departs from the reference" in r.stderr
    assert "1.11" in r.stderr
    r = subprocess.run([CLI, "--fasta-input", os.path.join(FIXTURES, "example.fasta"), "--pair-output",
                        str(tmp_path / "p.tsv")], capture_output=True, text=True, env=env)
    assert "exact-sums" not in r.stderr


def test_cli_weights_output_before_gpu_step(tmp_path):
    # the weights file is written before the all-pairs step (main.rs:161-164),
    # so it is checkable without a GPU: example.fasta lib.rs-derived weights.
    wpath = tmp_path / "w.tsv"
    r = subprocess.run([CLI, "--fasta-input", os.path.join(FIXTURES, "example.fasta"), "--pair-output",
                        str(tmp_path / "p.tsv"), "--weights-output", str(wpath)], capture_output=True, text=True)
    lines = wpath.read_text().splitlines()
    assert lines[0] == "Sequence_index\thk_weight"
    assert [l.split("\t")[1] for l in lines[1:]] == ["1.000", "0.300", "0.300", "0.300", "0.700"] + ["0.200"] * 5
    if not _gpu_present():
        assert r.returncode != 0 and "gfx950" in r.stderr
