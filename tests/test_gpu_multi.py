"""Multi-device contexts (wld_create_multi) and the CLI's --devices: the
reference's one all_weighted_ld_pairs call (lib.rs:578-684, main.rs:180-190)
sharded over G devices in one process.  G "virtual" devices are G contexts on
device 0 (one box has one GPU); the rows must be bit-identical to a single
context's, in the reference order, with progress reported on the calling
thread.
"""
import os
import subprocess
import threading

import numpy as np
import pytest

import _oracle as O
from conftest import CLI, FIXTURES, REPO
from test_gpu_parity import compare_rows, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def W():
    import weightedld_amd as W
    return W


def _same(a, b):
    for f in ("site_a", "site_b", "d", "d_prime", "r2"):
        x, y = getattr(a, f), getattr(b, f)
        assert len(x) == len(y), f
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32)), f


@pytest.mark.parametrize("G", [2, 3, 4])
@pytest.mark.parametrize("thr", [0.0, 0.02])
def test_group_rows_equal_single_context(W, G, thr):
    L, N = 1400, 600
    buf = synth(L, N, 40 + G)
    ss = W.SiteSet.from_buffer(buf)
    w = W.henikoff_weights(ss)
    single = W.Context(0)
    ref = W.all_weighted_ld_pairs(ss, w, thr, ctx=single)
    group = W.Context(devices=[0] * G)
    assert group.n_devices() == G
    seen, tids = [], set()

    def progress(n):
        seen.append(n)
        tids.add(threading.get_ident())

    got = W.all_weighted_ld_pairs(ss, w, thr, progress_report=progress, ctx=group)
    _same(got, ref)
    # lib.rs:584, then once per chunk with the count before it (lib.rs:670-674),
    # whichever member finished the chunk
    n_chunks = group.chunks(L)
    assert seen[0] == 0 and seen == sorted(seen) and len(seen) == 1 + n_chunks and seen[-1] < L * (L - 1) // 2
    assert tids == {threading.get_ident()}  # lib.rs:582's callback, on the calling thread
    st = group.stats()
    assert st["pairs"] == L * (L - 1) // 2 and st["rows"] == len(ref)
    if thr > 0:
        compare_rows(got, O.all_pairs(buf, w, np.float32(thr)), np.float32(thr), buf=buf, w=w)


def test_group_batches_and_options(W):
    # members split their shard into host batches (forced small) and take the
    # group's options; the result is still the single context's
    L, N = 1100, 300
    buf = synth(L, N, 77)
    w = np.random.default_rng(2).random(N).astype(np.float32) + 0.1
    single = W.Context(0)
    single.load(buf, w)
    ref = single.run_host(0.01)
    group = W.Context(devices=[0, 0, 0])
    group.set_option("host_batch_pairs", 70000)
    group.set_option("screen", 0)
    assert group.get_option("screen") == 0
    group.load(buf, w)
    _same(group.run_host(0.01), ref)


def test_group_rejects_single_device_calls(W):
    group = W.Context(devices=[0, 0])
    buf = synth(300, 100, 3)
    group.load(buf, np.ones(100, dtype=np.float32))
    for call in (lambda: group.run(0.0), lambda: group.dense(300), lambda: group.run_chunks_async(0.0)):
        with pytest.raises(W.WldError) as e:
            call()
        assert e.value.name == "WLD_E_STATE"
    # one pair on a group: its first device
    a, b = W.api.symbols_from_str("ACACACAA"), W.api.symbols_from_str("ACACACCA")
    r = W.single_weighted_ld_pair(a, None, b, None, np.ones(8, dtype=np.float32), ctx=group)
    r1 = W.single_weighted_ld_pair(a, None, b, None, np.ones(8, dtype=np.float32))
    assert r == r1


@pytest.mark.parametrize("devices", ["0,0", "0,0,0,0"])
def test_cli_devices_tsv_identical(tmp_path, devices):
    fasta = os.path.join(tmp_path, "s.fasta")
    buf = synth(700, 120, 5)
    with open(fasta, "w") as f:
        for k in range(buf.shape[1]):
            f.write(">s%d\n%s\n" % (k, "".join("ACGT-"[c] for c in buf[:, k])))
    outs = []
    for extra in ([], ["--devices", devices]):
        out = os.path.join(tmp_path, "p%d.tsv" % len(outs))
        r = subprocess.run([CLI, "--fasta-input", fasta, "--pair-output", out, "--r2-threshold", "0.01", *extra],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        outs.append(open(out).read())
    assert outs[0] == outs[1] and outs[0].count("\n") > 100


def test_cli_devices_fixture(tmp_path):
    out = os.path.join(tmp_path, "p.tsv")
    r = subprocess.run([CLI, "--fasta-input", os.path.join(FIXTURES, "t6_varsites_hk_ld.fasta"), "--pair-output", out,
                        "--devices", "0,0,0"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    r1 = subprocess.run([CLI, "--fasta-input", os.path.join(FIXTURES, "t6_varsites_hk_ld.fasta"), "--pair-output",
                         out + ".1"], capture_output=True, text=True, timeout=120)
    assert r1.returncode == 0 and open(out).read() == open(out + ".1").read()
