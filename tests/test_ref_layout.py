"""CPU check of the lib.rs-order index maps (pair_valu.hip): the lane-class
layout with transposed 16-position groups (ref_layout_kernel), the order in
which the f32-MFMA kernel consumes it (lane group g at step j of group grp
takes position 16 grp + 4 g + j), the order in which the per-pair chain
(ref_chain) walks it, and the scalar tail.  Each is replayed here in float32
and must give lib.rs's sums bit for bit: 8 lane sums over k = j (mod 8) below
8 floor(N/8), their ordered horizontal sum, then the tail (lib.rs:416-480)."""
import numpy as np
import pytest


def ref_layout(N):
    """Position -> sequence (-1 = padding), as ref_layout_kernel."""
    n8 = N // 8
    stages = (n8 + 63) // 64
    cls = stages * 64
    tail = 1 if N % 8 else 0
    NPr = 8 * cls + (64 if tail else 0) or 64
    seq = np.full(NPr, -1)
    for p in range(NPr):
        if p < 8 * cls:
            blk, tp = divmod(p, cls)
            t = (tp & ~15) | ((tp & 3) << 2) | ((tp >> 2) & 3)
            if t < n8:
                seq[p] = 8 * t + blk
        elif p - 8 * cls < N - 8 * n8:
            seq[p] = 8 * n8 + (p - 8 * cls)
    return seq, cls


def librs_sums(terms):
    """lib.rs's order for one of the four sums: terms[k] = w_k or 0."""
    N = len(terms)
    n8 = N // 8
    lanes = np.zeros(8, dtype=np.float32)
    for t in range(n8):
        for j in range(8):
            lanes[j] = np.float32(lanes[j] + terms[8 * t + j])
    tot = np.float32(0)
    for j in range(8):
        tot = np.float32(tot + lanes[j])
    for k in range(8 * n8, N):
        tot = np.float32(tot + terms[k])
    return tot


def mfma_order(terms, seq, cls, N):
    """The f32-MFMA kernel: per class, stages of 64 positions, groups grp,
    steps j, lane groups g (the MFMA's k) at position 16 grp + 4 g + j."""
    tot = np.float32(0)
    for c in range(8 if cls else 0):
        acc = np.float32(0)
        for k0 in range(c * cls, (c + 1) * cls, 64):
            for grp in range(4):
                for j in range(4):
                    for g in range(4):
                        s = seq[k0 + 16 * grp + 4 * g + j]
                        acc = np.float32(acc + (terms[s] if s >= 0 else np.float32(0)))
        tot = np.float32(tot + acc)
    for t in range(N - 8 * (N // 8)):
        tot = np.float32(tot + terms[seq[8 * cls + t]])
    return tot


def chain_order(terms, seq, cls, N):
    """ref_chain: 16-byte groups, element e = 4j + g at position 4g + j."""
    tot = np.float32(0)
    for c in range(8 if cls else 0):
        acc = np.float32(0)
        for q0 in range(c * cls, (c + 1) * cls, 16):
            for e in range(16):
                g, j = e & 3, e >> 2
                s = seq[q0 + 4 * g + j]
                acc = np.float32(acc + (terms[s] if s >= 0 else np.float32(0)))
        tot = np.float32(tot + acc)
    for t in range(N - 8 * (N // 8)):
        tot = np.float32(tot + terms[seq[8 * cls + t]])
    return tot


@pytest.mark.parametrize("N", [1, 7, 8, 9, 37, 300, 517, 1031])
def test_ref_layout_orders_equal_librs(N):
    rng = np.random.default_rng(N)
    seq, cls = ref_layout(N)
    real = seq[seq >= 0]
    assert sorted(real.tolist()) == list(range(N))  # every sequence exactly once
    for _ in range(3):
        w = (rng.random(N) * rng.choice([1e-3, 1.0, 1e3], size=N)).astype(np.float32)
        terms = np.where(rng.random(N) < 0.6, w, np.float32(0)).astype(np.float32)
        want = librs_sums(terms)
        assert mfma_order(terms, seq, cls, N).view(np.uint32) == want.view(np.uint32)
        assert chain_order(terms, seq, cls, N).view(np.uint32) == want.view(np.uint32)
