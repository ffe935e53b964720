"""The pair kernels' skip test (pair_common.hpp r2_bound_skip, compiled for
the host from the same source) against the f32 epilogue (lib.rs:482-520) on
adversarial inputs: a pair it skips must never pass r2 > thr when the
epilogue runs on the correctly rounded exact sums — including the
near-degenerate tables (a minor allele carrying ~1e-6 of the weight) where the
round-1 margin (1e-5 + 1e-4 thr below thr) skipped pairs that pass — and with
approximate sums (the one-plane screen: every 2x2 cell within R in total).
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO

U = 2.0 ** -24


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("bound") / "bound_check")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17", "-ffp-contract=off",
                    "-I", os.path.join(REPO, "include"), "-I", os.path.join(REPO, "weightedld_amd", "csrc"),
                    "-x", "hip", os.path.join(REPO, "tests", "cpp", "bound_check.cpp"), "-o", exe], check=True)

    def run(T, A, B, AB, R, thr, nonneg=True, f32=False, Tg=None, xy=False, fg=False, xy2=False):
        n = len(T)
        last = float(nonneg) if Tg is None else Tg
        rec = np.stack([np.asarray(x, np.float64) * np.ones(n) for x in (T, A, B, AB, R, thr, last)], 1)
        d = tmp_path_factory.mktemp("io")
        rec.tofile(str(d / "in.bin"))
        mode = (["f32xy2" if xy2 else "f32fg" if fg else "f32xy" if xy else "f32g"] if Tg is not None else
                ["f32"] if f32 else [])
        subprocess.run([exe, str(d / "in.bin"), str(d / "out.bin")] + mode, check=True)
        return np.fromfile(str(d / "out.bin"), dtype=np.uint8).astype(bool)
    return run


def f32_r2(T, SA, SB, SAB):
    """ld_epilogue's r2 on the f32-rounded sums (numpy float32, op for op)."""
    f = np.float32
    T, PA, PB, o3 = T.astype(f), SA.astype(f), SB.astype(f), SAB.astype(f)
    with np.errstate(all="ignore"):
        Pa, Pb = T - PA, T - PB
        o1 = PB - o3
        o2 = PA - o3
        o0 = Pa - o1
        PA, PB, Pa, Pb = PA / T, PB / T, Pa / T, Pb / T
        o0, o1, o2, o3 = o0 / T, o1 / T, o2 / T, o3 / T
        d = ((PA * PB - o3) + (Pa * Pb - o0) + (o2 - PA * Pb) + (o1 - Pa * PB)) / f(4)
        return d * d / (PA * Pa * PB * Pb)


def near_threshold_tables(rng, n, thr, scale=2.0 ** 34, window=3e-3):
    """Integer 2x2 tables with rare cells and exact r2 just below thr."""
    e = 10.0 ** rng.uniform(-6, -1, (3, n))
    n11, n10, n01 = np.floor(e[0] * scale), np.floor(e[1] * scale), np.floor(e[2] * scale)
    n00 = scale - n11 - n10 - n01
    T, A, B, AB = n11 + n10 + n01 + n00, n11 + n10, n11 + n01, n11
    num, den = A * B - AB * T, A * (T - A) * B * (T - B)
    r2 = num * num / den
    sel = (r2 < thr) & (r2 > thr * (1 - window))
    return T[sel], A[sel], B[sel], AB[sel]


def test_bound_sound_on_near_degenerate_tables(harness):
    rng = np.random.default_rng(7)
    viol_old = viol_new = skipped = total = 0
    for thr in (0.05, 0.1, 0.3):
        for _ in range(20):
            T, A, B, AB = near_threshold_tables(rng, 1_000_000, thr)
            passes = f32_r2(T, A, B, AB) > np.float32(thr)
            skip = harness(T, A, B, AB, 0.0, thr)
            num, den = A * B - AB * T, A * (T - A) * B * (T - B)
            old = (den > 0) & (num * num < (thr - (1e-5 + 1e-4 * thr)) * den)  # round 1's margin
            viol_new += int((skip & passes).sum())
            viol_old += int((old & passes).sum())
            skipped += int(skip.sum())
            total += len(T)
    assert total > 10_000 and skipped > 0.1 * total
    assert viol_new == 0
    assert viol_old > 0  # the round-1 margin was unsound on these tables


@pytest.mark.parametrize("nonneg", [True, False])
def test_bound_sound_with_screen_residuals(harness, nonneg):
    # approximate sums: cells perturbed by integers with sum |e_c| <= R
    rng = np.random.default_rng(11 + nonneg)
    viol = skipped = 0
    for it in range(30):
        n = 200_000
        scale = 2.0 ** rng.integers(12, 36)
        c = rng.random((4, n)) + (0.02 if it % 3 else 0.0)
        if it % 3 == 2:  # rare alleles
            eps = 10.0 ** rng.uniform(-5, -1, n)
            c[0] *= eps
            c[1] *= eps
        c = np.floor(c * scale)
        if not nonneg:  # cells may be negative (signed weights)
            c[rng.integers(0, 4, n), np.arange(n)] *= -0.01
            c = np.floor(c)
        T, A, B, AB = c.sum(0), c[0] + c[1], c[0] + c[2], c[0]
        thr = float(np.float32(rng.choice([0.01, 0.05, 0.2, 0.6])))
        R = np.floor(rng.choice([0.0, 1e-4, 1e-3, 1e-2]) * scale)
        e = rng.random((4, n)) * rng.choice([-1.0, 1.0], (4, n))
        e = np.trunc(e / np.maximum(np.abs(e).sum(0), 1e-12) * R * rng.random(n))
        h = c + e
        skip = harness(h.sum(0), h[0] + h[1], h[0] + h[2], h[0], R, thr, nonneg)
        with np.errstate(invalid="ignore"):
            passes = f32_r2(T, A, B, AB) > np.float32(thr)
        if nonneg:
            assert (c >= 0).all()
        viol += int((skip & passes).sum())
        skipped += int(skip.sum())
    assert viol == 0 and skipped > 0


def screen_tables(rng, n, scale, rare):
    """Nonnegative integer cells (top-plane sums, |T| <= 2^22) and screen
    residuals: approximate cells within R in total."""
    c = rng.random((4, n)) + 0.02
    if rare:
        eps = 10.0 ** rng.uniform(-4, -1, n)
        c[0] *= eps
        c[1] *= eps
    c = np.floor(c / c.sum(0) * scale)
    return c


@pytest.mark.parametrize("rare", [False, True])
def test_screen_f32_bound_sound_and_tight(harness, rare):
    # r2_screen_skip_f32 (the one-plane screen's per-pair test): never skips a
    # pair whose exact sums pass r2 > thr through the f32 epilogue, for any
    # approximation within R; and it skips nearly every pair the f64 test
    # skips (the screen kernel runs the f64 test on the pairs it leaves)
    rng = np.random.default_rng(23 + rare)
    viol = skipped = skipped64 = both = 0
    for it in range(24):
        n = 200_000
        scale = float(2 ** rng.integers(10, 22))
        c = screen_tables(rng, n, scale, rare)
        T, A, B, AB = c.sum(0), c[0] + c[1], c[0] + c[2], c[0]
        thr = float(np.float32(rng.choice([0.001, 0.01, 0.05, 0.2, 0.6])))
        R = rng.choice([0.0, 1e-4, 1e-3, 1e-2]) * scale * rng.random()
        e = rng.random((4, n)) * rng.choice([-1.0, 1.0], (4, n))
        e = np.trunc(e / np.maximum(np.abs(e).sum(0), 1e-12) * R * rng.random(n))
        h = c + e
        # near-threshold pairs: scale the off-diagonal so exact r2 sits at thr
        args = (h.sum(0), h[0] + h[1], h[0] + h[2], h[0], R, thr)
        s32 = harness(*args, f32=True)
        s64 = harness(*args)
        with np.errstate(invalid="ignore"):
            passes = f32_r2(T, A, B, AB) > np.float32(thr)
        viol += int((s32 & passes).sum())
        skipped += int(s32.sum())
        skipped64 += int(s64.sum())
        both += int((s32 & s64).sum())
    assert viol == 0
    assert skipped > 0
    # ordinary tables: the f32 form alone decides nearly all of them; with
    # marginals below 2^-12 of T it declines (the kernel's f64 test decides)
    assert skipped >= (0.6 if rare else 0.97) * skipped64, (skipped, skipped64)


@pytest.mark.parametrize("thr", [0.05, 0.1, 0.3])
def test_screen_f32_bound_sound_near_threshold(harness, thr):
    rng = np.random.default_rng(int(thr * 1000))
    viol = skipped = 0
    for _ in range(10):
        T, A, B, AB = near_threshold_tables(rng, 1_000_000, thr, scale=2.0 ** 22, window=0.05)
        passes = f32_r2(T, A, B, AB) > np.float32(thr)
        for R in (0.0, 1.0, 17.5):
            skip = harness(T, A, B, AB, R, thr, f32=True)
            viol += int((skip & passes).sum())
            skipped += int(skip.sum())
    assert viol == 0 and skipped > 0


@pytest.mark.parametrize("rare", [False, True])
def test_screen_launch_constants_sound(harness, rare):
    # the screen kernel's split form: E and 2^-12 Tb from a launch-wide Tg >= T
    # (Tg = 2 sum |top digits|), terms per pair.  With Tg = T it decides exactly
    # as r2_screen_skip_f32; with any larger Tg it never skips a pair whose
    # exact sums pass the f32 epilogue, and still skips most random tables.
    rng = np.random.default_rng(41 + rare)
    viol = skipped = same = total = 0
    for it in range(12):
        n = 200_000
        scale = float(2 ** rng.integers(10, 22))
        c = screen_tables(rng, n, scale, rare)
        T, A, B, AB = c.sum(0), c[0] + c[1], c[0] + c[2], c[0]
        thr = float(np.float32(rng.choice([0.001, 0.01, 0.05, 0.2, 0.6])))
        R = rng.choice([0.0, 1e-4, 1e-3, 1e-2]) * scale * rng.random()
        e = rng.random((4, n)) * rng.choice([-1.0, 1.0], (4, n))
        e = np.trunc(e / np.maximum(np.abs(e).sum(0), 1e-12) * R * rng.random(n))
        h = c + e
        args = (h.sum(0), h[0] + h[1], h[0] + h[2], h[0], R, thr)
        with np.errstate(invalid="ignore"):
            passes = f32_r2(T, A, B, AB) > np.float32(thr)
        eq = harness(*args, Tg=h.sum(0))
        same += int((eq == harness(*args, f32=True)).sum())
        total += n
        for f in (1.0, 1.3, 4.0):
            Tg = float(h.sum(0).max()) * f
            s = harness(*args, Tg=Tg)
            viol += int((s & passes).sum())
            skipped += int(s.sum())
    assert viol == 0
    assert same == total
    assert skipped > 0


@pytest.mark.parametrize("thr", [0.05, 0.3])
def test_screen_launch_constants_near_threshold(harness, thr):
    rng = np.random.default_rng(int(thr * 1000) + 7)
    viol = 0
    for _ in range(6):
        T, A, B, AB = near_threshold_tables(rng, 1_000_000, thr, scale=2.0 ** 22, window=0.05)
        passes = f32_r2(T, A, B, AB) > np.float32(thr)
        for R in (0.0, 1.0, 17.5):
            for Tg in (float(T.max()), float(T.max()) * 2.0):
                viol += int((harness(T, A, B, AB, R, thr, Tg=Tg) & passes).sum())
    assert viol == 0


@pytest.mark.parametrize("rare", [False, True])
def test_screen_accumulator_form_sound(harness, rare):
    # r2_screen_terms_xy (the screen kernel's form, from the X/Y accumulators):
    # sound for any Tg >= T, and it decides like the (T, A, B, AB) form except
    # where the differently rounded numerator lands on the other side.
    rng = np.random.default_rng(53 + rare)
    viol = diff = total = 0
    for it in range(12):
        n = 200_000
        scale = float(2 ** rng.integers(10, 21))
        c = screen_tables(rng, n, scale, rare)
        T, A, B, AB = c.sum(0), c[0] + c[1], c[0] + c[2], c[0]
        thr = float(np.float32(rng.choice([0.001, 0.01, 0.05, 0.2, 0.6])))
        R = rng.choice([0.0, 1e-4, 1e-3, 1e-2]) * scale * rng.random()
        e = rng.random((4, n)) * rng.choice([-1.0, 1.0], (4, n))
        e = np.trunc(e / np.maximum(np.abs(e).sum(0), 1e-12) * R * rng.random(n))
        h = 2 * (c + e)  # doubled sums: X = (T + B) / 2 etc. are integers
        args = (h.sum(0), h[0] + h[1], h[0] + h[2], h[0], 2 * R, thr)
        with np.errstate(invalid="ignore"):
            passes = f32_r2(T, A, B, AB) > np.float32(thr)
        for f in (1.0, 2.0):
            Tg = float(h.sum(0).max()) * f
            sx = harness(*args, Tg=Tg, xy=True)
            sg = harness(*args, Tg=Tg)
            viol += int((sx & passes).sum())
            diff += int((sx != sg).sum())
            total += n
    assert viol == 0
    assert diff <= total // 10000, (diff, total)


@pytest.mark.parametrize("thr", [0.05, 0.3])
def test_screen_accumulator_form_near_threshold(harness, thr):
    rng = np.random.default_rng(int(thr * 1000) + 11)
    viol = 0
    for _ in range(6):
        T, A, B, AB = near_threshold_tables(rng, 1_000_000, thr, scale=2.0 ** 21, window=0.05)
        passes = f32_r2(T, A, B, AB) > np.float32(thr)
        for R in (0.0, 1.0, 17.5):
            for Tg in (2 * float(T.max()), 4 * float(T.max())):
                viol += int((harness(2 * T, 2 * A, 2 * B, 2 * AB, 2 * R, thr, Tg=Tg, xy=True) & passes).sum())
    assert viol == 0


@pytest.mark.parametrize("form", ["fg", "xy2"])
@pytest.mark.parametrize("rare", [False, True])
def test_screen_fp6_dual_form_sound(harness, rare, form):
    # r2_screen_terms_fg (the fp6 screen's form, from the e2m3 / e3m2 readings
    # of the b codes; exact marginals, R on the accumulators' grid, marginals
    # tested against mloc as the screen's per-lane minimum): never skips a pair
    # whose exact sums pass the f32 epilogue, for any Tg >= T, and decides like
    # the X/Y form but for pairs on the edge of a rounding.
    rng = np.random.default_rng(67 + rare)
    viol = diff = more = total = skipped = 0
    for it in range(12):
        n = 200_000
        scale = float(2 ** rng.integers(10, 21))
        c = screen_tables(rng, n, scale, rare)
        T, A, B, AB = c.sum(0), c[0] + c[1], c[0] + c[2], c[0]
        thr = float(np.float32(rng.choice([0.001, 0.01, 0.05, 0.2, 0.6])))
        R = rng.choice([0.0, 1e-4, 1e-3, 1e-2]) * scale * rng.random()
        e = rng.random((4, n)) * rng.choice([-1.0, 1.0], (4, n))
        e = np.trunc(e / np.maximum(np.abs(e).sum(0), 1e-12) * R * rng.random(n))
        h = 2 * (c + e)
        args = (h.sum(0), h[0] + h[1], h[0] + h[2], h[0], 2 * R, thr)
        with np.errstate(invalid="ignore"):
            passes = f32_r2(T, A, B, AB) > np.float32(thr)
        for f in (1.0, 2.0):
            Tg = float(h.sum(0).max()) * f
            sf = harness(*args, Tg=Tg, **{form: True})
            sx = harness(*args, Tg=Tg, xy=True)
            viol += int((sf & passes).sum())
            diff += int((sf != sx).sum())
            more += int((sf & ~sx).sum())
            skipped += int(sf.sum())
            total += n
    assert viol == 0
    assert skipped > total // 4
    print("%s vs xy: %d of %d decisions differ, %d of them skips only %s makes" % (form, diff, total, more, form))
    assert more == 0  # never skips a pair the X/Y form keeps
    assert diff <= total // 1000, (diff, total)


@pytest.mark.parametrize("form", ["fg", "xy2"])
@pytest.mark.parametrize("thr", [0.05, 0.3])
def test_screen_fp6_dual_form_near_threshold(harness, thr, form):
    rng = np.random.default_rng(int(thr * 1000) + 13)
    viol = 0
    for _ in range(6):
        T, A, B, AB = near_threshold_tables(rng, 1_000_000, thr, scale=2.0 ** 21, window=0.05)
        passes = f32_r2(T, A, B, AB) > np.float32(thr)
        for R in (0.0, 1.0, 17.5):
            for Tg in (2 * float(T.max()), 4 * float(T.max())):
                viol += int((harness(2 * T, 2 * A, 2 * B, 2 * AB, 2 * R, thr, Tg=Tg, **{form: True}) & passes).sum())
    assert viol == 0
