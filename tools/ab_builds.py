#!/usr/bin/env python3
"""A/B timing of experimental library builds (tools/build_variant.sh), one
child process per (round, build), interleaved.  Prints per-build median
pair-kernel ms (HIP events) at a bench config with the default kernel."""
import argparse
import json
import os
import statistics
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(path, config, reps, thr, unweighted=False):
    sys.path.insert(0, REPO)
    import torch  # noqa: F401
    import weightedld_amd._lib as L
    L.LIB_PATH = os.path.abspath(path)
    import bench
    import weightedld_amd as W
    if "," in config:  # custom shape "N,L,thr"
        N, Ls, thr0 = int(config.split(",")[0]), int(config.split(",")[1]), float(config.split(",")[2])
    else:
        N, Ls, thr0, _ = bench.CONFIGS[config]
    thr = thr0 if thr is None else thr
    buf = bench.ld_blocks(Ls, N) if os.environ.get("WLD_AB_DATA") == "ldblocks" else bench.synth(Ls, N)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    if unweighted:
        w = np.ones(N, dtype=np.float32)
    if os.environ.get("WLD_AB_WEIGHTS") == "2pl":  # two active digit planes (1 and 2)
        w = np.where(np.random.default_rng(3).random(N) < 0.5, 1.0, 3 / 256).astype(np.float32)
    ctx = W.Context(0, W.KERNEL_MFMA)
    for kv in filter(None, os.environ.get("WLD_AB_OPTS", "").split(";")):  # name=path@WLD_AB_OPTS=opt=v;opt=v
        k, v = kv.split("=", 1)
        ctx.set_option(k, int(v))
    ctx.load(buf, w)
    shard = int(os.environ.get("WLD_AB_SHARD", "1"))  # rank 0's 1/K shard of the chunk sequence
    lb, le = W.Context.shard_chunks(Ls, shard, 0) if shard > 1 else (0, 0)
    run = (lambda t: ctx.run_chunks(t, lb, le)) if shard > 1 else ctx.run
    run(thr)
    import ctypes
    lib = W.lib()
    st = None
    if hasattr(lib, "wld_debug_stamps"):
        st = (ctypes.c_ulonglong * 8)()
        lib.wld_debug_stamps(st, 1)
    t, rows, ts = [], 0, []
    for _ in range(reps):
        rows = run(thr)
        sx = ctx.stats()
        t.append(sx["pair_kernel_ms"])
        ts.append(sx.get("screen_ms", 0.0))
    out = {"ms": t, "rows": rows, "screen_ms": sorted(ts)[len(ts) // 2], "cand": ctx.stats()["candidate_tiles"],
           "screened": ctx.stats()["screened"]}
    ops = 8.0 * ctx.stats()["mfma_planes"] * ((N + 63) // 64 * 64) * (Ls * (Ls - 1) / 2)
    out["tops"] = ops / (sorted(t)[len(t) // 2] * 1e-3) / 1e12
    if st is not None:
        lib.wld_debug_stamps(st, 0)
        n = max(st[5], 1)
        out["stamps_per_wave"] = {"prologue": st[0] / n, "loop": st[1] / n, "epilogue": (st[2] - st[0] - st[1]) / n,
                                  "compaction": st[3] / n, "waves": st[5]}
    print(json.dumps(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--child")
    ap.add_argument("--config", default="c4")
    ap.add_argument("--thr", type=float)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--unweighted", action="store_true")
    ap.add_argument("builds", nargs="*", help="name=path/to/libweightedld.so")
    a = ap.parse_args()
    if a.child:
        return child(a.child, a.config, a.reps, a.thr, a.unweighted)
    res = {}
    for _ in range(a.rounds):
        for b in a.builds:
            name, path = b.split("=", 1)
            env = dict(os.environ)
            if "@" in path:  # name=path@VAR=value[,VAR=value]
                path, kvs = path.split("@", 1)
                for kv in kvs.split(","):
                    k, v = kv.split("=", 1)
                    env[k] = v
            cmd = [sys.executable, __file__, "--child", path, "--config", a.config, "--reps", str(a.reps)]
            if a.unweighted:
                cmd += ["--unweighted"]
            if a.thr is not None:
                cmd += ["--thr", str(a.thr)]
            out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
            if out.returncode:
                print(json.dumps({"build": name, "rc": out.returncode, "err": out.stderr[-800:]}), flush=True)
                if out.returncode < 0 or out.returncode >= 124:
                    sys.exit(out.returncode if out.returncode > 0 else 1)
                continue
            r = json.loads(out.stdout.strip().splitlines()[-1])
            res.setdefault(name, {"ms": [], "rows": r["rows"]})["ms"] += r["ms"]
            res[name].setdefault("screen_ms", []).append(r.get("screen_ms", 0.0))
            print(json.dumps({"build": name, "median_ms": statistics.median(r["ms"]), "rows": r["rows"], "tops": r["tops"],
                              "screen_ms": r.get("screen_ms"), "cand": r.get("cand"),
                              "screened": r.get("screened"), "stamps": r.get("stamps_per_wave")}), flush=True)
    for name, r in res.items():
        print(json.dumps({"build": name, "median_ms": statistics.median(r["ms"]), "min_ms": min(r["ms"]),
                          "screen_ms": statistics.median(r.get("screen_ms", [0.0])), "rows": r["rows"],
                          "n": len(r["ms"])}))


if __name__ == "__main__":
    main()
