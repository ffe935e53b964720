"""Device pre-pass (wld_load_filtered, prepass.hip) against the oracle and the
host restatement of main.rs:139-156: the kept-site map equals the oracle's
is_site_of_interest mask (lib.rs:309-338, wldo_is_site_of_interest), the
Henikoff weights equal the oracle's on the kept buffer bit for bit
(lib.rs:340-380, wldo_henikoff_weights), and the rows computed from them are
identical to the host path's (wld_siteset_filter_sites_of_interest +
wld_henikoff_weights + wld_load)."""
import os

import numpy as np
import pytest

import _oracle as O  # checker only
from conftest import FIXTURES
from test_gpu_parity import synth

pytestmark = pytest.mark.gpu

FASTAS = ["example.fasta", "t2_henikoff_complex1.fasta", "t3_henikoff_complex2.fasta", "t4_weights1_ld0.fasta",
          "t5_weights1_ld0.25.fasta", "t6_varsites_hk_ld.fasta"]


@pytest.fixture(scope="module")
def W():
    import weightedld_amd as W
    return W


def host_path(W, ss, params, unweighted):
    kept = ss.filter_sites_of_interest(*params)
    w = np.ones(ss.n_seqs(), dtype=np.float32) if unweighted else W.henikoff_weights(kept)
    return kept, w


def check_oracle(dev, buf, params, unweighted):
    """The device pre-pass against the oracle itself: kept sites = the
    oracle's mask, weights = the oracle's Henikoff weights of the kept buffer
    (unit weights when unweighted, main.rs:150-153), bit for bit."""
    buf = np.minimum(buf, 5).astype(np.uint8)  # Symbol codes are 0..5 (the product clamps larger bytes to Unknown)
    mask = O.site_mask(buf, *params)
    assert np.array_equal(dev.site_map(), np.nonzero(mask)[0].astype(np.uint64))
    ref_w = np.ones(buf.shape[1], dtype=np.float32) if unweighted else O.henikoff_weights(buf[mask])
    wd = dev.weights()
    assert np.array_equal(wd.view(np.uint32), ref_w.view(np.uint32)), (wd[:5], ref_w[:5])


def check_equal(W, buf, params=(0.8, 0.02, 0.5), unweighted=False, thr=0.0, kernel=None):
    ss = W.SiteSet.from_buffer(buf)
    kept, w = host_path(W, ss, params, unweighted)
    kernel = W.KERNEL_AUTO if kernel is None else kernel
    dev = W.Context(0, kernel)
    n = dev.load_filtered(buf, *params, unweighted=unweighted)
    check_oracle(dev, buf, params, unweighted)
    assert n == kept.n_sites()
    sm = kept.site_map if kept.site_map is not None else np.arange(kept.n_sites(), dtype=np.uint64)
    assert np.array_equal(dev.site_map(), sm)
    wd = dev.weights()
    assert np.array_equal(wd.view(np.uint32), w.view(np.uint32)), (wd[:5], w[:5])
    if n == 0:
        return
    host = W.Context(0, kernel)
    host.load(kept.buffer, w, site_map=sm)
    na, nb = dev.run(thr), host.run(thr)
    assert na == nb
    ra, rb = dev.rows(), host.rows()
    for f in ("site_a", "site_b", "d", "d_prime", "r2"):
        x, y = getattr(ra, f), getattr(rb, f)
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32)), f


@pytest.mark.parametrize("name", FASTAS)
@pytest.mark.parametrize("unweighted", [False, True])
def test_prepass_fixtures(W, name, unweighted):
    ss = W.read_fasta(os.path.join(FIXTURES, name))
    check_equal(W, ss.buffer, unweighted=unweighted)


@pytest.mark.parametrize("L,N,seed,unknown", [(300, 200, 1, 0.0), (513, 333, 2, 0.03), (257, 1000, 3, 0.2),
                                              (100, 40000, 4, 0.01), (3, 8193, 5, 0.05), (7, 8192, 7, 0.1),
                                              (1030, 130, 6, 0.02), (1, 65, 8, 0.1)])
def test_prepass_synthetic(W, L, N, seed, unknown):
    # Unknown symbols exercise the Henikoff fill term; N > 8192 exceeds a wave's
    # LDS row stage (site_stats_kernel), L % 4 != 0 a partial site workgroup,
    # N % 64 != 0 a partial sequence workgroup and n_kept % 256 != 0 a partial
    # site block (henikoff_seq_kernel)
    check_equal(W, synth(L, N, seed, unknown=unknown))


def test_prepass_filter_edges(W):
    # sites failing each clause of is_site_of_interest: too few ACGT, monomorphic,
    # minor fraction out of range, all Unknown; plus a code > Unknown (clamped)
    rng = np.random.default_rng(7)
    N = 120
    buf = synth(60, N, 8)
    buf[0] = 4                      # all missing -> acgt too low
    buf[1] = 2                      # monomorphic
    buf[2, :] = 0
    buf[2, :1] = 1                  # minor fraction 1/120 < 0.02
    buf[3] = 5                      # all Unknown
    buf[4, ::3] = 4                 # 33% missing -> acgt = 80 < ceil(0.8*120)=96
    buf[5, :] = np.where(rng.random(N) < 0.5, 0, 3)
    buf[6, 5] = 9                   # clamped to Unknown
    check_equal(W, buf)
    check_equal(W, buf, params=(0.5, 0.0, 1.0))
    check_equal(W, buf, params=(0.95, 0.1, 0.4), unweighted=True)


@pytest.mark.parametrize("kern", ["valu", "mfma"])
def test_prepass_kernels_and_threshold(W, kern):
    k = W.KERNEL_VALU if kern == "valu" else W.KERNEL_MFMA
    check_equal(W, synth(700, 300, 12, unknown=0.02), thr=0.01, kernel=k)


def test_prepass_vcf(W):
    ss = W.read_vcf(os.path.join(FIXTURES, "t7_1000genome.vcf"))
    check_equal(W, ss.buffer)
    check_equal(W, ss.buffer, unweighted=True)


def test_prepass_device_input_and_composed_map(W):
    import torch
    buf = synth(400, 250, 13, unknown=0.01)
    ss = W.SiteSet.from_buffer(buf)
    kept, w = host_path(W, ss, (0.8, 0.02, 0.5), False)
    d = torch.from_numpy(buf).cuda()
    ctx = W.Context(0)
    pos = np.arange(400, dtype=np.uint64) * 10 + 7  # e.g. VCF POS
    n = ctx.load_filtered_device(d.data_ptr(), 400, 250, site_map=pos)
    assert n == kept.n_sites()
    assert np.array_equal(ctx.site_map(), pos[kept.site_map.astype(np.int64)])
    assert np.array_equal(ctx.weights().view(np.uint32), w.view(np.uint32))
    ctx.run(0.0)
    rows = ctx.rows()
    assert set(np.unique(rows.site_a)).issubset(set(pos.astype(np.uint32)))


@pytest.mark.parametrize("name", FASTAS)
@pytest.mark.parametrize("unweighted", [False, True])
def test_cli_gpu_prepass_same_output(tmp_path, name, unweighted):
    # --gpu-prepass must write byte-identical pair and weight TSVs
    import subprocess
    from test_gpu_parity import CLI
    outs = []
    for flag in ([], ["--gpu-prepass"]):
        pairs, wts = tmp_path / ("p%d.tsv" % len(flag)), tmp_path / ("w%d.tsv" % len(flag))
        cmd = [CLI, "--fasta-input", os.path.join(FIXTURES, name), "--pair-output", str(pairs),
               "--weights-output", str(wts), "--r2-threshold", "0.0"] + flag
        if unweighted:
            cmd.append("--unweighted")
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
        if name == "t1_henikoff_paper.fasta":
            assert r.returncode == 101
            return
        assert r.returncode == 0, r.stderr
        outs.append((pairs.read_bytes(), wts.read_bytes()))
    assert outs[0] == outs[1]


@pytest.mark.parametrize("config", ["c2", "c4", "c5"])
def test_prepass_bench_workloads_vs_oracle(W, config):
    """The full bench inputs (BASELINE configs 2, 4 and 5: up to 50,000 sites
    x 5,000 sequences), random and (C4) linkage blocks with Unknown symbols
    sprinkled in: the device's kept-site map and Henikoff weights equal the
    oracle's bit for bit."""
    import bench
    N, L, _, _ = bench.CONFIGS[config]
    bufs = [bench.synth(L, N)]
    if config == "c4":
        ld = bench.ld_blocks(L, N)
        rng = np.random.default_rng(11)
        ld[rng.random(ld.shape) < 0.01] = 5  # Unknown: the Henikoff fill term
        bufs.append(ld)
    for buf in bufs:
        dev = W.Context(0)
        n = dev.load_filtered(buf, 0.8, 0.02, 0.5)
        assert n > 0
        check_oracle(dev, buf, (0.8, 0.02, 0.5), False)
        dev.close()
