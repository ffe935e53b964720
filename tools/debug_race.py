#!/usr/bin/env python3
"""GPU diagnostic over raw ctypes (works with any build of the C ABI):
repeated wld_run of one input must give bit-identical rows, equal to the
oracle's f32 values within 1e-5.  Unit weights (one digit plane) by default.
    python tools/debug_race.py LIB [--weights ones|henikoff] [--runs K] [--thr T ...]"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--weights", default="ones")
    ap.add_argument("--runs", type=int, default=6)
    ap.add_argument("--thr", type=float, nargs="*", default=[0.002])
    ap.add_argument("--L", type=int, default=3000)
    ap.add_argument("--N", type=int, default=2000)
    ap.add_argument("--opt", nargs="*", default=[], help="option_id=value (wld_set_option)")
    ap.add_argument("--dense", action="store_true", help="compare wld_dense matrices across runs instead")
    a = ap.parse_args()
    import _oracle as O
    from test_gpu_parity import synth
    buf = np.ascontiguousarray(synth(a.L, a.N, 8))
    if a.weights == "ones":
        w = np.ones(a.N, dtype=np.float32)
    elif a.weights == "two":  # two nonzero digit planes
        w = np.where(np.random.default_rng(3).random(a.N) < 0.5, 1.0, 3 / 256).astype(np.float32)
    else:
        import weightedld_amd as W
        w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    lib = C.CDLL(os.path.abspath(a.lib))
    lib.wld_last_error.restype = C.c_char_p
    ctx = C.c_void_p()
    assert lib.wld_create(0, C.byref(ctx)) == 0, lib.wld_last_error()
    for kv in a.opt:
        k, v = kv.split("=")
        assert lib.wld_set_option(ctx, int(k), C.c_int64(int(v))) == 0, lib.wld_last_error()
    assert lib.wld_load(ctx, buf.ctypes.data_as(C.c_void_p), C.c_size_t(a.L), C.c_size_t(a.N), None,
                        w.ctypes.data_as(C.c_void_p)) == 0, lib.wld_last_error()
    if a.dense:
        L = a.L
        first = None
        for run in range(a.runs):
            d, dp, r2 = (np.zeros(L * L, np.float32) for _ in range(3))
            v = np.zeros(L * L, np.uint8)
            assert lib.wld_dense(ctx, *(x.ctypes.data_as(C.c_void_p) for x in (d, dp, r2, v))) == 0
            if first is None:
                first = d.copy()
                print("dense run 0", flush=True)
            else:
                diff = np.nonzero(first.view(np.uint32) != d.view(np.uint32))[0]
                print("dense run %d: %d values differ from run 0 %s" % (
                    run, len(diff), [(int(i // L), int(i % L), float(first[i]), float(d[i])) for i in diff[:3]]),
                    flush=True)
                # group by (a, 16-column block of b): which rows / column blocks
                groups = {}
                for i in diff:
                    a_, b_ = int(i // L), int(i % L)
                    groups.setdefault((a_, b_ // 16), []).append(b_ % 16)
                for (a_, bb), cols in sorted(groups.items())[:12]:
                    print("   a %d (a%%64 %d) b-block %d (b%%64 block %d): cols %s" % (
                        a_, a_ % 64, bb, (bb * 16) % 64 // 16, sorted(cols)), flush=True)
                    # where else in the tile (run 0) the wrong values occur
                    b_ = bb * 16 + sorted(cols)[0]
                    wrong = d[a_ * L + b_]
                    ta0, tb0 = a_ // 64 * 64, b_ // 64 * 64
                    tile = first.reshape(L, L)[ta0:ta0 + 64, tb0:tb0 + 64]
                    hits = np.argwhere(tile.view(np.uint32) == np.float32(wrong).view(np.uint32))
                    print("      wrong %r right %r; equal to run-0 tile cells (da, db) %s" % (
                        float(wrong), float(first[a_ * L + b_]),
                        [(int(x) - (a_ - ta0), int(y) - (b_ - tb0)) for x, y in hits[:8]]), flush=True)
        return
    for thr in a.thr:
        ref = O.all_pairs(buf, w, np.float32(thr))
        key = {(int(x), int(y)): i for i, (x, y) in enumerate(zip(ref["site_a"], ref["site_b"]))}
        first = None
        for run in range(a.runs):
            n = C.c_uint64()
            assert lib.wld_run(ctx, C.c_float(thr), 0, 0, C.byref(n)) == 0, lib.wld_last_error()
            n = n.value
            sa, sb = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
            d, dp, r2 = np.zeros(n, np.float32), np.zeros(n, np.float32), np.zeros(n, np.float32)
            assert lib.wld_rows_copy(ctx, *(x.ctypes.data_as(C.c_void_p) for x in (sa, sb, d, dp, r2))) == 0
            idx = np.array([key.get((int(x), int(y)), -1) for x, y in zip(sa, sb)])
            ok = idx >= 0
            bad = np.zeros(n, bool)
            bad[ok] = np.abs(d[ok] - ref["d"][idx[ok]]) > 1e-5
            same = None
            if first is None:
                first = d.copy()
            else:
                same = len(first) == len(d) and np.array_equal(first.view(np.uint32), d.view(np.uint32))
            ex = [(int(sa[i]), int(sb[i]), float(d[i]), float(ref["d"][idx[i]])) for i in np.nonzero(bad)[0][:3]]
            if hasattr(lib, "wld_debug_lds_mismatch"):
                mm = (C.c_ulonglong * 4)()
                lib.wld_debug_lds_mismatch(mm)
                print("  lds mismatches (cumulative): blocks %d digits %d lanes12-14 %d checks %d" % tuple(mm))
            print("thr %g run %d rows %d (ref %d) not-in-ref %d bad-d %d same-as-run0 %s %s" % (
                thr, run, n, len(ref["d"]), int((~ok).sum()), int(bad.sum()), same, ex), flush=True)


if __name__ == "__main__":
    main()
