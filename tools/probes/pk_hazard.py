#!/usr/bin/env python3
"""Packed-f32 probe ("Packed-f32 code generation").

With hipcc's SLP vectorizer on, the pair kernels' f32 epilogue is emitted with
v_pk_add_f32 / v_pk_mul_f32, and the one-plane MFMA kernel's dense and
prefilter modes gave wrong d/d'/r2 in lanes 48-63 of a few tiles per run.
This probe runs that failing case (unit weights: one digit plane; 3000 sites
x 2000 sequences; dense stats and an unscreened prefilter run) on library
variants that differ only in how pair_mfma.hip was compiled
(tools/build_variant.sh):
  pk_base      -fno-slp-vectorize (the shipped flags)           reference
  pk_slp       SLP on (packed f32 in the epilogue)
  pk_slp_padK  SLP on + -mllvm -amdgpu-snop-padding=K (s_nop K, K+1 wait states,
               before EVERY instruction), K = 1..4
and counts, per run, the values that differ from pk_base bit for bit and the
accumulator rows (a mod 16) they fall on.  If padding every instruction with
wait states removes the errors, the packed code is right and a wait state is
missing (a pipeline hazard the compiler does not pad); if the errors stay,
it is not a hazard between instructions.

    python tools/probes/pk_hazard.py [--reps 3]      (GPU box; prints one JSON line per run)
    python tools/probes/pk_hazard.py --small         (640 sites: one workgroup per CU, 40 runs)
"""
import argparse
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
VARIANTS = ["pk_base", "pk_slp", "pk_slp_pad1", "pk_slp_pad2", "pk_slp_pad3", "pk_slp_pad4"]
L, N = 3000, 2000
# --small: 640 sites = 55 tiles on 256 CUs, one workgroup per CU (no
# co-resident waves on the SIMD), REPS dense runs in one process
SMALL_L, SMALL_REPS = 640, 40


def child(variant, out_npz, small=False):
    sys.path.insert(0, REPO)
    import torch  # noqa: F401  (one HIP runtime: torch's)
    import weightedld_amd._lib as WL
    WL.LIB_PATH = os.path.join(REPO, "build", "exp", variant, "libweightedld.so")
    import bench
    import weightedld_amd as W
    Ls = SMALL_L if small else L
    buf = bench.synth(Ls, N)
    w = np.ones(N, dtype=np.float32)
    ctx = W.Context(0, W.KERNEL_MFMA, ref_sums=False)
    ctx.load(buf, w)
    assert ctx.stats()["mfma_planes"] == 1
    if small:  # stack the repetitions' dense stats along a new axis
        runs = [ctx.dense(Ls) for _ in range(SMALL_REPS)]
        np.savez(out_npz, r2=np.stack([r[2] for r in runs]))
        return
    d, dp, r2, valid = ctx.dense(L)
    ctx.set_option("screen", 0)  # the unscreened one-plane prefilter kernel
    ctx.run(0.001)
    rows = ctx.rows()
    np.savez(out_npz, d=d, dp=dp, r2=r2, valid=valid, ra=rows.site_a, rb=rows.site_b, rd=rows.d, rdp=rows.d_prime,
             rr2=rows.r2)


def compare(ref, got):
    iu = np.triu_indices(L, 1)
    res = {"dense_values": 3 * len(iu[0])}
    bad_rows = np.zeros(16, dtype=np.int64)
    nbad = 0
    for f in ("d", "dp", "r2"):
        a, b = ref[f][iu], got[f][iu]
        bad = (a.view(np.uint32) != b.view(np.uint32)) & ~(np.isnan(a) & np.isnan(b))
        nbad += int(bad.sum())
        np.add.at(bad_rows, iu[0][bad] % 16, 1)
    res["dense_bad"] = nbad
    res["dense_bad_by_a_mod_16"] = bad_rows.tolist()
    same_rows = len(ref["ra"]) == len(got["ra"]) and np.array_equal(ref["ra"], got["ra"]) and \
        np.array_equal(ref["rb"], got["rb"])
    res["prefilter_rows_ref_gpu"] = [int(len(ref["ra"])), int(len(got["ra"]))]
    if same_rows:
        res["prefilter_bad"] = int(sum((ref[f].view(np.uint32) != got[f].view(np.uint32)).sum()
                                       for f in ("rd", "rdp", "rr2")))
    else:
        res["prefilter_bad"] = "row sets differ"
    return res


def compare_small(ref, got):
    bad = (ref["r2"].view(np.uint32) != got["r2"].view(np.uint32)) & ~(np.isnan(ref["r2"]) & np.isnan(got["r2"]))
    iu = np.triu_indices(SMALL_L, 1)
    b = bad[:, iu[0], iu[1]]
    rows = np.zeros(16, dtype=np.int64)
    np.add.at(rows, np.nonzero(b)[1] * 0 + iu[0][np.nonzero(b)[1]] % 16, 1)
    return {"small_L": SMALL_L, "reps": SMALL_REPS, "r2_values": int(b.size), "r2_bad": int(b.sum()),
            "bad_by_a_mod_16": rows.tolist()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--child", nargs=2)
    ap.add_argument("--small", action="store_true")
    a = ap.parse_args()
    if a.child:
        child(*a.child, small=a.small)
        return
    tmp = os.environ.get("TMPDIR", "/tmp")
    if a.small:
        ref_path = os.path.join(tmp, "pk_ref_small.npz")
        subprocess.run([sys.executable, __file__, "--small", "--child", "pk_base", ref_path], check=True, timeout=300)
        ref = np.load(ref_path)
        for v in ("pk_slp", "pk_slp_pad1"):
            p = os.path.join(tmp, "pk_small_%s.npz" % v)
            subprocess.run([sys.executable, __file__, "--small", "--child", v, p], check=True, timeout=300)
            print(json.dumps({"variant": v, **compare_small(ref, np.load(p))}), flush=True)
        return
    ref_path = os.path.join(tmp, "pk_ref.npz")
    subprocess.run([sys.executable, __file__, "--child", "pk_base", ref_path], check=True, timeout=300)
    ref = np.load(ref_path)
    for rep in range(a.reps):
        for v in VARIANTS:
            p = os.path.join(tmp, "pk_%s.npz" % v)
            subprocess.run([sys.executable, __file__, "--child", v, p], check=True, timeout=300)
            print(json.dumps({"variant": v, "rep": rep, **compare(ref, np.load(p))}), flush=True)


if __name__ == "__main__":
    main()
