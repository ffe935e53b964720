#!/usr/bin/env python3
"""Headline benchmark: LD site-pairs/s at N=2000 sequences x L=20000 sites (BASELINE config 4).

A "step" is one all_weighted_ld_pairs pass (lib.rs:578-684) over the whole
synthetic alignment: the pair kernel over this rank's chunk-range shard, the
reference-order assembly of the rows with r2 > 0.05 and, for N>1, their RCCL
gather to rank 0.  Inputs (site codes + weights) are resident in HBM before
the timed region.  Total work is fixed as N grows (strong scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4|c2|c5]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU)

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts its
own N ranks (one process per GPU, RANK/LOCAL_RANK/WORLD_SIZE set) before
anything touches torch or the GPU, and relays rank 0's line; under torchrun
WORLD_SIZE must equal --gpus.  Rank 0 prints ONE JSON line.  The CPU baseline
(rank 0 at N=1, after the timed region; null at N>1) is the C restatement of the
lib.rs simd path (oracle/wld_oracle.c, "port"), threaded like rayon over
256x256 chunks, timed on a bounded sample of the same workload.
"""
import argparse
import collections
import json
import os
import socket
import subprocess
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
METRIC = "LD site-pairs/sec at N=2000 seq × L=20000 var sites; 1/2/4/8 GPU; %HBM roofline"
CONFIGS = {
    # name: (n_seqs, n_sites, r2_threshold, description)
    "c2": (500, 2000, 0.0, "BASELINE config 2: synthetic 500 seq x 2000 sites, r2_threshold=0.0"),
    "c4": (2000, 20000, 0.05, "BASELINE config 4: synthetic 2000 seq x 20000 sites, r2_threshold=0.05"),
    "c5": (5000, 50000, 0.05, "BASELINE config 5: synthetic 5000 seq x 50000 sites, r2_threshold=0.05"),
}
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak (spec)
I8_MFMA_PEAK_TOPS = 5000.0  # dense i8 MFMA = 2x bf16 dense 2.5 PF (MI355X_MICROARCH.md Matrix cores)
# dense fp6/fp4 block-scaled MFMA (v_mfma_scale_f32_16x16x128_f8f6f4 with e2m3 x
# e2m1 operands: 4x bf16 per clock, MI355X_MICROARCH.md Matrix cores FP6 row)
FP6_MFMA_PEAK_TFLOPS = 10000.0
F32_VALU_PEAK_TFLOPS = 157.3  # FP32 vector peak (spec) = f32-input MFMA peak


def synth(L, N, seed=0x5EED, block=4096):
    """bench_weighted_pair_ld.rs:8-28 distribution, seeded: per site a major !=
    minor from ACGT; each sequence '-' w.p. 0.10, major 0.60, else minor."""
    rng = np.random.Generator(np.random.PCG64(seed))
    maj = rng.integers(0, 4, size=L)
    mnr = (maj + rng.integers(1, 4, size=L)) % 4
    out = np.empty((L, N), dtype=np.uint8)
    for s0 in range(0, L, block):
        s1 = min(L, s0 + block)
        u = rng.random((s1 - s0, N), dtype=np.float32)
        out[s0:s1] = np.where(u < 0.1, 4, np.where(u < 0.7, maj[s0:s1, None], mnr[s0:s1, None]))
    return out


def ld_blocks(L, N, seed=0x1DB1, min_block=20, max_block=200, p_missing=0.1, p_mut=0.02):
    """Linkage-structured alignment (--data ldblocks): consecutive blocks of
    20-200 sites; in each block every sequence copies one of 3-8 founder
    haplotypes (random proportions), every site gives each founder a major
    or minor symbol (a random 0/1 pattern, minor frequency 0.2-0.5 among
    founders' carriers), each copy mutates w.p. p_mut and is '-' w.p.
    p_missing.  Pairs inside a block are in strong LD (many rows at 0.05),
    pairs across blocks near r2 ~ 1/N."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = np.empty((L, N), dtype=np.uint8)
    s0 = 0
    while s0 < L:
        s1 = min(L, s0 + int(rng.integers(min_block, max_block + 1)))
        H = int(rng.integers(3, 9))
        founder = rng.choice(H, size=N, p=rng.dirichlet(np.ones(H)))
        n = s1 - s0
        maj = rng.integers(0, 4, size=n)
        mnr = (maj + rng.integers(1, 4, size=n)) % 4
        pat = rng.random((n, H)) < rng.uniform(0.2, 0.5, size=(n, 1))  # founder carries the minor
        pat[np.arange(n), rng.integers(0, H, size=n)] ^= ~pat.any(axis=1)  # every site polymorphic
        allele = pat[:, founder] ^ (rng.random((n, N), dtype=np.float32) < p_mut)
        col = np.where(allele, mnr[:, None], maj[:, None])
        out[s0:s1] = np.where(rng.random((n, N), dtype=np.float32) < p_missing, 4, col)
        s0 = s1
    return out


def vcf_like(L, n_hap=5008, seed=0x1000, p_missing=0.002, p_rare=0.5):
    """1000-Genomes-like biallelic haplotypes (BASELINE config 3 at scale):
    a Kingman coalescent over n_hap haplotypes, sites = mutations dropped on
    its branches in proportion to their lengths (allele-frequency spectrum
    ~1/k, LD as the tree makes it: sites on one branch in perfect LD, nested
    clades partial), plus a fraction p_rare of recent variants carried by 1-4
    random haplotypes (the excess of singletons and doubletons a growing
    population shows: about 60% of sites have an allele count <= 4).
    Symbols as handle_vcf makes them (WeightedLD.py:348-363): 0 ref, 1 alt,
    4 missing ('.')."""
    rng = np.random.Generator(np.random.PCG64(seed))
    n = n_hap
    lineages = list(range(n))
    members = [np.array([i], dtype=np.int32) for i in range(n)]
    born = [0.0] * n
    length = [0.0] * n
    t = 0.0
    while len(lineages) > 1:
        k = len(lineages)
        t += rng.exponential(2.0 / (k * (k - 1)))
        i, j = sorted(rng.choice(k, size=2, replace=False))
        a, b = lineages[i], lineages[j]
        length[a] = t - born[a]
        length[b] = t - born[b]
        members.append(np.concatenate([members[a], members[b]]))
        born.append(t)
        length.append(0.0)
        lineages[j] = lineages[-1]
        lineages.pop()
        lineages[i] = len(members) - 1
    p = np.asarray(length) / np.sum(length)
    branch = rng.choice(len(members), size=L, p=p)
    out = np.zeros((L, n), dtype=np.uint8)
    rare = rng.random(L) < p_rare
    for s, br in enumerate(branch):
        if rare[s]:
            out[s, rng.choice(n, size=int(rng.integers(1, 5)), replace=False)] = 1
        else:
            out[s, members[br]] = 1
    out[rng.random((L, n), dtype=np.float32) < p_missing] = 4
    return out


def planted_ld(L, N, seed=0x91A7, n_tiles=400, max_per_tile=3):
    """The headline's seeded background (synth) with planted linkage: the
    workload where the screen must reject nearly every tile yet keep the few
    that hold rows.  About n_tiles 64x64 tiles each get 1..max_per_tile site
    pairs (a, b), b's column a copy of a's with a fraction p of its entries
    replaced by a permutation of a's (p in {0 .. 0.78}: r2 from 1 down to about
    the 0.05 threshold, some just below it).  Every planted site is used once.
    The tiles include, deliberately: diagonal tiles (rows of both parities,
    i.e. first halves of tile-pair entries and single entries, tile 0 and the
    padded last tile), the padded last tile column (single entries), tiles
    (ta, tb) with tb even and odd (both halves of a tile pair), the rest
    uniform over the triangle (every XCD queue); a deliberately chosen tile's
    first pair has p <= 0.3, so it holds a row.  Returns (buf, planted) with
    planted = [(a, b, p)]."""
    buf = synth(L, N)
    rng = np.random.Generator(np.random.PCG64(seed))
    T = (L + 63) // 64
    tiles = []
    diag = set(rng.choice(np.arange(1, T - 1), size=min(T - 2, 40), replace=False).tolist()) | {0, 1, T - 2, T - 1}
    tiles += [(t, t) for t in sorted(diag)]
    tiles += [(int(t), T - 1) for t in rng.choice(T - 1, size=min(T - 1, 30), replace=False)]
    for parity in (0, 1):
        k = 0
        while k < 30:
            ta = int(rng.integers(0, T - 2))
            tb = int(rng.integers(ta + 1, T - 1))
            if tb % 2 == parity:
                tiles.append((ta, tb))
                k += 1
    while len(set(tiles)) < n_tiles:
        ta, tb = sorted(int(x) for x in rng.integers(0, T, size=2))
        tiles.append((ta, tb))
    deliberate = set(tiles)
    # the deliberate tiles first, in the order chosen (the padded last tile's
    # 32 sites go to the diagonal tile before the last column), then the rest
    tiles = list(dict.fromkeys(tiles))
    used = np.zeros(L, dtype=bool)
    planted = []
    levels = np.array([0.0, 0.1, 0.2, 0.3, 0.45, 0.6, 0.7, 0.75, 0.78])

    def free_site(t, exclude=-1):
        lo, hi = 64 * t, min(L, 64 * t + 64)
        cand = [s for s in range(lo, hi) if not used[s] and s != exclude]
        return int(rng.choice(cand)) if cand else -1

    for ta, tb in tiles:
        for k in range(int(rng.integers(1, max_per_tile + 1))):
            a = free_site(ta)
            if a < 0:
                break
            used[a] = True
            b = free_site(tb)
            if b < 0:
                used[a] = False
                break
            used[b] = True
            a, b = min(a, b), max(a, b)
            # (a deliberately chosen tile's first pair well above the threshold)
            p = float(rng.choice(levels[:4] if k == 0 and (ta, tb) in deliberate else levels))
            col = buf[a].copy()
            m = rng.random(N) < p
            col[m] = rng.permutation(buf[a])[m]
            buf[b] = col
            planted.append((a, b, p))
    return buf, planted


def pairs_in_rows(L, rb, re_):
    a0, a1 = min(L, rb * 256), min(L, re_ * 256)
    return (a1 - a0) * (L - 1) - (a1 - 1 + a0) * (a1 - a0) // 2 if a1 > a0 else 0


def chunk_pairs(L, i):
    n = (L + 255) // 256
    rf = int(((8 * i + 1) ** 0.5 - 1) / 2)
    while (rf + 1) * (rf + 2) // 2 <= i:
        rf += 1
    while rf * (rf + 1) // 2 > i:
        rf -= 1
    row = n - rf - 1
    col = row + i - rf * (rf + 1) // 2
    sa = min(L, row * 256 + 256) - row * 256
    sb = min(L, col * 256 + 256) - col * 256
    return sa * (sa - 1) // 2 if row == col else sa * sb


def cpu_baseline(buf, w, thr, target_s=15.0, max_s=30.0):
    """Times the oracle (C restatement of the lib.rs simd path) on the same
    workload: all of it when that fits in max_s seconds of CPU work, else the
    first chunks in triu order, sized to ~target_s seconds."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import _oracle as O  # checker / baseline only

    O.use_native()  # gcc -O3 -march=native on the measuring host
    threads, share = host_cpu_share()
    L = buf.shape[0]
    n = (L + 255) // 256
    nchunks = n * (n + 1) // 2

    last = {}

    def run(k):
        t0 = time.perf_counter()
        r = O.all_pairs(buf, w, thr, n_threads=threads, chunk_lo=0, chunk_hi=k)
        dt = time.perf_counter() - t0
        last.update(rows=r, chunks=k)
        return r["pairs"], dt

    # calibrate on ~1/16 of the chunks (enough work to amortise thread start-up)
    k = min(nchunks, max(4 * threads, nchunks // 16))
    p, t = run(k)
    rate = p / max(t, 1e-9)
    total = L * (L - 1) // 2
    if total / rate <= max_s:
        k2 = nchunks
        what = "the whole workload (%d reference chunks)" % nchunks
    else:
        want = rate * target_s
        k2, acc = 0, 0
        while k2 < nchunks and acc < want:
            acc += chunk_pairs(L, k2)
            k2 += 1
        k2 = max(k2, 1)
        what = "the first %d of %d reference chunks (256x256, triu order) of the same workload" % (k2, nchunks)
    p, t = run(k2)
    return last["rows"], last["chunks"], {"value": p / t, "unit": "site-pairs/s", "cores": threads, "kind": "port",
            "sample": "%s = %d pairs in %.1f s; C restatement of the lib.rs simd path (8-lane f32, rayon-style "
                      "chunk scheduling), gcc -O3 -march=native" % (what, p, t), "host_cpus": share}


def fp6_planted_check(W, dev_index, L, N, thr):
    """The headline screen where it can fail: the same size
    and threshold as the timed workload, with planted linkage (planted_ld:
    ~770 rows over ~380 tiles on every XCD queue, both halves of tile-pair
    entries, single entries, diagonal and padded tiles), the fp6 screen forced
    (WLD_OPT_SCREEN_FP6 2) and in auto, each pass's rows against the oracle's
    bit for bit, with the candidate counts.  Outside the timed region."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import _oracle as O  # checker only
    O.use_native()
    buf, planted = planted_ld(L, N)
    w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
    t0 = time.perf_counter()
    ref = O.all_pairs(buf, w, np.float32(thr), n_threads=host_cpu_share()[0])
    oracle_s = time.perf_counter() - t0
    out = {"data": "bench.planted_ld (seeded background + %d planted pairs)" % len(planted), "thr": thr,
           "oracle_rows": int(len(ref["r2"])),
           "tiles_holding_rows": len(set(zip((ref["site_a"] // 64).tolist(), (ref["site_b"] // 64).tolist()))),
           "oracle_s": oracle_s}
    for mode, opt in (("forced", 2), ("auto", None)):
        c = W.Context(dev_index)
        if opt is not None:
            c.set_option("screen_fp6", opt)
        c.load(buf, w)
        n = c.run(thr)
        st = c.stats()
        g = c.rows()
        equal = n == len(ref["r2"]) and all(
            np.array_equal(np.asarray(getattr(g, f)).astype(np.uint32), np.asarray(ref[f]).astype(np.uint32))
            for f in ("site_a", "site_b")) and all(
            np.array_equal(np.asarray(getattr(g, f), dtype=np.float32).view(np.uint32),
                           np.asarray(ref[f], dtype=np.float32).view(np.uint32)) for f in ("d", "d_prime", "r2"))
        out[mode] = {"gpu_rows": n, "equal": bool(equal), "screen_fp6": st["screen_fp6"],
                     "candidate_tiles": st["candidate_tiles"], "candidate_blocks": st["candidate_blocks"],
                     "tiles": st["tiles"], "pair_kernel_ms": st["pair_kernel_ms"]}
        c.close()
    out["equal"] = out["forced"]["equal"] and out["auto"]["equal"] and out["forced"]["screen_fp6"] == 1
    return out


def host_cpu_share():
    """The threads the CPU baseline runs on: every CPU this process may use
    (rayon's default is all logical cores, lib.rs:635-637) — its affinity set,
    capped by a cgroup CPU quota when one is set (a leased share of a larger
    host: os.cpu_count() then counts CPUs the process cannot get).  Returns
    (threads, the figures that decided it)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):  # cgroup v2: "<quota> <period>" or "max <period>"
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
        except (OSError, ValueError):
            pass
    if quota is None:
        try:  # cgroup v1
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    threads = aff if quota is None else max(1, min(aff, int(quota + 0.5)))
    why = ("affinity set" if quota is None or threads == aff else "cgroup CPU quota (below the affinity set)")
    return threads, {"os_cpu_count": os.cpu_count(), "affinity": aff, "cgroup_quota_cpus": quota,
                     "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"), "threads_from": why}


def load_traffic(config, kernel):
    path = os.path.join(REPO, "profiles", "traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
        return t.get("%s/%s" % (config, kernel))
    except Exception:
        return None


def launch_ranks(n, argv):
    """--gpus N > 1 without a launcher: N child ranks of this script (one per
    GPU, LOCAL_RANK = RANK), started before this process imports torch or
    touches a GPU.  Rank 0's stdout (the JSON line) is relayed to stdout, the
    other ranks' to stderr.  A rank that fails stops the others; returns the
    first nonzero exit status (0 when all succeed)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs, relays = [], []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WLD_BENCH_SPAWNED="1")
        p = subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + list(argv), env=env,
                             stdout=subprocess.PIPE, text=True, bufsize=1)
        procs.append(p)

        def relay(src, dst):
            for line in src:
                dst.write(line)
                dst.flush()

        t = threading.Thread(target=relay, args=(p.stdout, sys.stdout if r == 0 else sys.stderr), daemon=True)
        t.start()
        relays.append(t)
    rc, kill_at = 0, None
    live = set(range(n))
    while live:
        for r in sorted(live):
            c = procs[r].poll()
            if c is None:
                continue
            live.discard(r)
            if c != 0 and rc == 0:
                rc = c
                print("bench.py: rank %d exited with status %d; stopping the other ranks" % (r, c), file=sys.stderr)
                for k in live:
                    procs[k].terminate()
                kill_at = time.time() + 20.0
        if kill_at is not None and time.time() > kill_at:
            for k in live:
                procs[k].kill()
            kill_at = None
        time.sleep(0.05)
    for t in relays:
        t.join(timeout=10)
    return rc if rc >= 0 else 128 - rc


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--settle-s", type=float, default=0.3,
                    help="untimed back-to-back steps before the warmup while the GPU clock settles (seconds)")
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--kernel", default="auto", choices=["auto", "valu", "mfma"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--unweighted", action="store_true", help="unit weights (main.rs:150-153 --unweighted)")
    ap.add_argument("--wide-weights", action="store_true",
                    help="Henikoff weights with every 10th scaled by 2^-8 (range ~2^-8: the 4-plane kernel)")
    ap.add_argument("--thr", type=float, help="override the config's r2 threshold (non-headline lines)")
    ap.add_argument("--rehearse-dist", action="store_true",
                    help="at N=1: run the N>1 step path (RCCL group of one, ShardStep/pipelined steps)")
    ap.add_argument("--tile-rows", action="store_true",
                    help="plain (a-tile, b-tile) launch order instead of the XCD-aware one (WLD_OPT_TILE_ORDER 1; same rows)")
    ap.add_argument("--pipe-depth", type=int, default=0, metavar="D",
                    help="contexts of the pipelined step loop, D - 1 steps in flight (default: 3 for the N>1 "
                         "step path, where unserialized screens take rank 0's 1/8 shard of C4 from 0.142 to "
                         "0.118 ms/step, archive/profiles_r01_r03/r03j/; 2 at N=1, where three measured equal, archive/profiles_r01_r03/r03q/)")
    ap.add_argument("--rehearse-shard", type=int, default=0, metavar="K",
                    help="with --rehearse-dist: run rank 0's shard of a K-way split (the per-rank work at "
                         "N=K; value counts that shard's pairs); a rehearsal line, never the headline")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="one step at a time (N=1: no second context; N>1: one ShardStep at a time)")
    ap.add_argument("--no-screen", action="store_true",
                    help="every tile with every weight-digit plane (WLD_OPT_SCREEN 0; same rows)")
    ap.add_argument("--no-prefilter", action="store_true",
                    help="every pair through the f32 epilogue (WLD_OPT_PREFILTER 0, implies --no-screen; same rows)")
    ap.add_argument("--data", default="random", choices=["random", "ldblocks"],
                    help="random: the seeded bench_weighted_pair_ld.rs distribution (the headline); ldblocks: the "
                         "same size with linkage blocks of 20-200 sites (many rows, candidate tiles)")
    ap.add_argument("--exact-sums", action="store_true",
                    help="exact sums rounded once (WLD_OPT_REF_SUMS 0) instead of the default, lib.rs's own f32 "
                         "summation order (rows bit-identical to lib.rs)")
    ap.add_argument("--collectives", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (default): RCCL over xGMI, one GPU per rank; gloo: counts and rows exchanged as host "
                         "tensors, ranks may share a GPU (rank r on device r mod the visible count: the multi-rank "
                         "test of the launcher on a one-GPU box, never a headline line)")
    ap.add_argument("--counts", default="auto", choices=["auto", "shm", "collective"],
                    help="N>1 step path: how the ranks exchange each step's row counts.  shm: through host shared "
                         "memory once each rank's pass has completed (weightedld_amd.dist.HostCountExchange; ranks "
                         "on one host); collective: an all_gather queued behind the pass on the device (RCCL, or "
                         "gloo with --collectives gloo); auto (default): shm when every rank is on this host.  "
                         "The rows always travel by the collective backend")
    ap.add_argument("--check-steps", type=int, default=0, metavar="K",
                    help="after the timed region, K more steps whose gathered rows rank 0 compares with the "
                         "oracle's (every row and bit, in reference order)")
    args = ap.parse_args()
    args.ref_sums = not args.exact_sums

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: start the N ranks here, before torch or the GPU is touched
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d (launch with --nproc-per-node equal to --gpus)" %
                         (args.gpus, world))

    import torch
    import torch.distributed as dist

    host_coll = args.collectives == "gloo"
    n_dev = torch.cuda.device_count()
    if n_dev == 0:
        raise SystemExit("bench.py: rank %d of %d: no GPU visible" % (rank, world))
    if not host_coll and local_rank >= n_dev:
        raise SystemExit("bench.py: rank %d needs GPU %d but %d are visible (one GPU per rank over RCCL)" %
                         (rank, local_rank, n_dev))
    dev_index = local_rank % n_dev
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    # small control collectives (settle-step count, max-over-ranks times):
    # device tensors over RCCL, host tensors over gloo
    cdev = torch.device("cpu") if host_coll else device
    dist_on = world > 1 or args.rehearse_dist  # the N>1 step path (a group of one when rehearsing)
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29571")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        if host_coll:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)

    sys.path.insert(0, REPO)
    import weightedld_amd as W

    N, L, thr, desc = CONFIGS[args.config]
    if args.thr is not None and args.thr != thr:
        thr = args.thr
        desc += " (r2_threshold overridden to %g)" % thr
    buf = synth(L, N) if args.data == "random" else ld_blocks(L, N)
    t0 = time.perf_counter()
    ss = W.SiteSet.from_buffer(buf)
    kept = ss.filter_sites_of_interest()  # host pre-pass (lib.rs:309-338, main.rs:139)
    weights = W.henikoff_weights(kept)  # host pre-pass (lib.rs:340-380)
    if args.unweighted:
        weights = np.ones(N, dtype=np.float32)
    if args.wide_weights:
        weights = weights.copy()
        weights[::10] *= np.float32(2.0 ** -8)
    prepass_ms = (time.perf_counter() - t0) * 1e3
    assert kept.n_sites() == L  # the synthetic distribution keeps every site
    torch.ones(1024, device=device).sum().item()  # CUDA context + allocator up before timing H2D
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d_buf = torch.from_numpy(buf).to(device)
    d_w = torch.from_numpy(weights).to(device)
    torch.cuda.synchronize()
    h2d_ms = (time.perf_counter() - t0) * 1e3

    kernel = {"auto": W.KERNEL_AUTO, "valu": W.KERNEL_VALU, "mfma": W.KERNEL_MFMA}[args.kernel]
    # the same pre-pass on the device from the resident raw
    # buffer (filter + Henikoff + encode), checked bit for bit against the host's
    pre = W.Context(dev_index, kernel)
    dev_ms = []
    for _ in range(3):
        assert pre.load_filtered_device(d_buf.data_ptr(), L, N, unweighted=args.unweighted) == L
        dev_ms.append(pre.stats()["load_ms"])
    if not args.wide_weights:
        assert np.array_equal(pre.weights().view(np.uint32), weights.view(np.uint32))
    pre.close()
    created = []  # every context of the run, closed explicitly at the end (newest first)

    def new_ctx():
        c = W.Context(dev_index, kernel)
        created.append(c)
        if args.no_screen or args.no_prefilter:
            c.set_option("screen", 0)
        if args.no_prefilter:
            c.set_option("prefilter", 0)
        if args.tile_rows:
            c.set_option("tile_order", 1)
        c.set_option("ref_sums", 0 if args.exact_sums else 1)
        # WLD_BENCH_OPTS="name=v;name=v": library options for A/B lines (never the headline's)
        for kv in filter(None, os.environ.get("WLD_BENCH_OPTS", "").split(";")):
            k, v = kv.split("=")
            c.set_option(k.strip(), int(v))
        c.load_device(d_buf.data_ptr(), L, N, d_w.data_ptr())
        return c

    ctx = new_ctx()
    load_ms = ctx.stats()["load_ms"]
    # contiguous run of the reference chunk sequence, balanced by pairs (weightedld_amd/dist.py)
    cb, ce = ctx.shard_chunks(L, world, rank)
    if args.rehearse_dist and args.rehearse_shard > 1:
        cb, ce = ctx.shard_chunks(L, args.rehearse_shard, 0)

    from weightedld_amd import dist as wdist

    gms = []
    # N>1: the shard's pair kernel and row count on the library's stream, the
    # RCCL count all_gather ordered after them on that stream, one host wait;
    # rows (if any) then gathered to rank 0 in reference order (shards
    # concatenate in descending rank order: chunk rows descend)
    shard_step = None  # (set below: the pipeline's first step when there is one)
    # N>1 timed steps: two contexts on the same resident inputs, step i's
    # kernel queued on the device behind step i-1's while step i-1's count
    # exchange / host read / row gather complete (PipelinedShardStep)
    # Pipelining doubles the contexts' operand footprint (two fragment copies of
    # 2 LP NP bytes each): only when both fit the 256 MB Infinity Cache (C4:
    # 2 x 81 MB); at C5 (2 x 500 MB) the alternating contexts measured 2% slower
    LP, NP = -(-L // 256) * 256, -(-N // 64) * 64
    pipelined = not args.no_pipeline and 2 * LP * NP <= 128 << 20
    pipe = None
    # N>1: three contexts, step i's screen may overlap step i-1's; N=1: two,
    # queued back to back with wld_run_after (WLD_PIPE_SERIALIZE / --pipe-depth
    # select the others)
    depth = args.pipe_depth or (3 if dist_on else 2)
    # N=1 "auto" (default): both orders are timed on the warm contexts after
    # the clock settle, interleaved, and the faster one runs the timed steps
    # (profiles/r06i/: free screens C4 0.543 against 0.558 ms/step and C2
    # 0.101 against 0.122, but LD blocks 1.220 against 1.186, where two
    # contexts' i8 operand images, 2 x 160 MB, exceed the Infinity Cache)
    serialize = os.environ.get("WLD_PIPE_SERIALIZE", "0" if dist_on else "auto")
    serialize_trials = None  # N=1 auto: {mode: [ms/step of each trial]}
    ctxs1 = None  # N=1: the contexts of the pipelined loop
    if not dist_on and pipelined:
        ctxs1 = [ctx] + [new_ctx() for _ in range(max(2, depth) - 1)]
        if serialize == "stream":  # every context on the first one's stream (wld_set_stream)
            for c in ctxs1[1:]:
                c.set_stream(ctx)
    xchg = None  # N>1: the row counts through host shared memory (--counts)
    if dist_on and args.counts != "collective":
        hosts = [None] * world
        if world > 1:
            dist.all_gather_object(hosts, socket.gethostname())
        one_host = world == 1 or len(set(hosts)) == 1
        if args.counts == "shm" and not one_host:
            raise SystemExit("bench.py: --counts shm needs every rank on one host")
        if one_host:
            xchg = wdist.HostCountExchange(rank, world)
    if dist_on and pipelined:
        pipe = wdist.PipelinedShardStep([ctx] + [new_ctx() for _ in range(max(2, depth) - 1)], rank, world,
                                        device,
                                        # 0 (default): step i's screen may start while step i-1's runs, so
                                        # a shard's last round of tiles overlaps the next step's first and
                                        # no cross-queue event wait (~20 us) sits between them; "pair":
                                        # step i's pair kernel waits on the device for step i-1's screen
                                        # (wld_run_after); 1: for step i-1's whole run (archive/profiles_r01_r03/r02pc/,
                                        # archive/profiles_r01_r03/r03i/)
                                        serialize_kernels={"0": False, "1": True}.get(serialize, "pair"),
                                        host_collectives=host_coll, counts=xchg)
    if dist_on:
        # single steps on ctx (stats sampling, unscreened and checked steps) go
        # through the pipeline's own step object for ctx: one stream per context
        shard_step = pipe.steps[0] if pipe is not None else wdist.ShardStep(ctx, rank, world, device,
                                                                              host_collectives=host_coll,
                                                                              counts=xchg)

    def nrows(res):
        return int(res[1].shape[1]) if res is not None and res[1] is not None else 0

    def step():
        if not dist_on:
            return ctx.run_chunks(thr, cb, ce)
        _, rows = shard_step(thr, cb, ce)
        return int(rows.shape[1]) if rows is not None else 0

    # steps stay in flight after a step with rows too: its gather is queued
    # behind its scan on the device (C2 0.157 -> 0.135 ms/step, LD blocks
    # 1.350 -> 1.305, profiles/r04g/); WLD_PIPE_DRAIN_ROWS=1 drains the
    # pipeline after such a step first (rounds 1-3)
    drain_rows = os.environ.get("WLD_PIPE_DRAIN_ROWS", "0") != "0"

    def run_steps(k):
        if ctxs1 is not None:
            # N=1 pipelined: step i on context i % D (D-buffered rows), up to
            # D - 1 steps in flight; the host completes the oldest step
            # (wld_run_wait) while the newer ones run.  Step i's screen may
            # start while step i-1's runs (WLD_PIPE_SERIALIZE=pair: queued
            # behind it with wld_run_after).
            pend, r = collections.deque(), 0
            for i in range(k):
                c = ctxs1[i % len(ctxs1)]
                if len(pend) == len(ctxs1) or (drain_rows and r > 0 and pend):
                    while pend and (len(pend) == len(ctxs1) or (drain_rows and r > 0)):
                        r = pend.popleft().run_wait()
                if pend and serialize in ("pair", "stream"):
                    c.run_after(pend[-1])  # this pair kernel queued behind the previous one (device wait)
                c.run_chunks_async(thr, cb, ce)
                pend.append(c)
            while pend:
                r = pend.popleft().run_wait()
            return r
        if pipe is None:
            r = 0
            for _ in range(k):
                r = step()
            return r
        for _ in range(k):
            pipe.submit(thr, cb, ce)
        return nrows(pipe.drain())

    # Clock settle (untimed, before the warmup): back-to-back steps for about
    # settle_s seconds.  The pair kernel's time falls over the first ~30
    # launches as the clock settles (rocprofv3 trace of `--steps 20 --warmup
    # 5`, archive/profiles_r01_r03/r03c/: a C4 screen launch 1.07 -> 0.90 ms), so a short
    # warmup would time the ramp, not the kernel.  Every rank runs the same
    # number of steps (their collectives pair up).
    settle_steps = 0
    if args.settle_s > 0:
        t1 = time.perf_counter()
        run_steps(3)
        torch.cuda.synchronize()
        per = (time.perf_counter() - t1) / 3
        settle_steps = int(np.ceil(args.settle_s / max(per, 1e-4)))
        if dist_on:
            t = torch.tensor([settle_steps], dtype=torch.int64, device=cdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            settle_steps = int(t.item())
        run_steps(settle_steps)
    if serialize == "auto":
        serialize = "pair"
        if ctxs1 is not None:
            # a trial = about settle_s / 6 of steps (at least 4) in one order
            n_trial = max(4, settle_steps // 6)
            serialize_trials = {"pair": [], "0": []}
            for _ in range(2):
                for m in ("pair", "0"):
                    serialize = m
                    torch.cuda.synchronize()
                    t1 = time.perf_counter()
                    run_steps(n_trial)
                    torch.cuda.synchronize()
                    serialize_trials[m].append((time.perf_counter() - t1) * 1e3 / n_trial)
            serialize = min(serialize_trials, key=lambda m: sum(serialize_trials[m]))
    run_steps(args.warmup)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rows = run_steps(args.steps)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # per-launch HIP-event times of the same steps, sampled after the timed
    # region so that reading them adds nothing to it
    kms, oms, sms, cand, cblk, cpairs = [], [], [], [], [], []
    for _ in range(min(args.steps, 20)):
        tg = time.perf_counter()
        step()
        st = ctx.stats()
        kms.append(st["pair_kernel_ms"])
        oms.append(st["order_ms"])
        sms.append(st["screen_ms"])
        cand.append(st["candidate_tiles"])
        cblk.append(st["candidate_blocks"])
        cpairs.append(st["candidate_pairs"])
        gms.append((time.perf_counter() - tg) * 1e3 - st["pair_kernel_ms"])
    # 0 none, 1 i8 one-plane screen, 3 two-plane screen, 4 exact candidate pairs
    screen_kind = ctx.stats()["screened"]
    screened = bool(screen_kind)
    fp6 = screen_kind == 1 and bool(ctx.stats()["screen_fp6"])  # the one-plane screen on fp6 x fp4 MFMA
    n_tiles = ctx.stats()["tiles"]
    # the same steps without the screen (every tile, every plane; same rows),
    # reported alongside: a few sequential runs after the timed region
    unscreened_ms = None
    if dist_on:  # every rank runs the same steps (their collectives pair up), whatever its own policy chose
        t = torch.tensor([int(screened)], dtype=torch.int64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        screened_any = bool(t.item())
    else:
        screened_any = screened
    if screened_any:
        ctx.set_option("screen", 0)
        ums = []
        for _ in range(5):
            step()
            ums.append(ctx.stats()["pair_kernel_ms"])
        ctx.set_option("screen", 1)
        unscreened_ms = float(np.mean(ums[1:])) if screened else None
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        km = torch.tensor([float(np.mean(kms)), float(np.mean(sms))], dtype=torch.float64, device=cdev)
        dist.all_reduce(km, op=dist.ReduceOp.MAX)
        kernel_ms, screen_ms = float(km[0].item()), float(km[1].item())
    else:
        kernel_ms, screen_ms = float(np.mean(kms)), float(np.mean(sms))
    st = ctx.stats()
    kern_name = "mfma" if st["kernel"] == W.KERNEL_MFMA else "valu"
    planes = st["mfma_planes"]

    # --check-steps: K more steps through the same step path (pipelined
    # contexts and the row gather at N>1); rank 0 keeps every step's rows
    checked = []
    if args.check_steps > 0:
        if not dist_on:
            for _ in range(args.check_steps):
                ctx.run_chunks(thr, cb, ce)
                g = ctx.rows()
                checked.append({f: np.array(getattr(g, f)) for f in wdist.ROW_FIELDS})
        else:
            res = []
            if pipe is not None:
                for _ in range(args.check_steps):
                    r = pipe.submit(thr, cb, ce)
                    if r is not None:
                        res.append(r)
                res += pipe.drain_all()
            else:
                res = [shard_step(thr, cb, ce) for _ in range(args.check_steps)]
            if rank == 0:
                checked = [wdist.unpack_rows(g) for _, g in res]
    torch.cuda.synchronize()

    def close_all():
        # the step streams first (their work done), then the contexts, newest
        # first, while torch and the HIP runtime are up (not at interpreter exit)
        if pipe is not None:
            pipe.close()
        if shard_step is not None:
            shard_step.close()
        for c in reversed(created):
            c.close()
        if xchg is not None:
            xchg.close()

    if dist_on:
        # no collective after this: the other ranks leave, so that rank 0's
        # CPU baseline runs with no rank polling beside it
        dist.destroy_process_group()
    if rank != 0:
        close_all()
        return

    total_pairs = L * (L - 1) // 2
    shard_pairs = ctx.pairs_in_chunks(L, cb, ce)
    if args.rehearse_dist and args.rehearse_shard > 1:
        total_pairs = shard_pairs  # one rank's shard of a K-way split, timed alone
        desc += " (rehearsal: rank 0's shard of %d)" % args.rehearse_shard
    value = total_pairs * args.steps / elapsed
    # Roofline of the dominant kernel: ALGORITHMIC work per
    # launch, SURVEY 8(d)'s 4 masked multiply-adds per (pair, sequence) =
    # 8 N ops per pair, over the launch's HIP-event time.  Screened runs: the
    # dominant kernel is the one-plane screen, which evaluates every pair of
    # the shard (its bound, from one digit plane of every sequence); the
    # candidate launch recomputes the few tiles it cannot reject.
    alg_ops = shard_pairs * 8.0 * N
    # the f32 kernel ran every tile: the f32 fallback, or the reference order
    # without a screen in front (thresholds <= 0, --no-screen)
    f32_path = kern_name == "valu" or (args.ref_sums and not screened)
    if not f32_path:
        # the dominant kernel's peak: dense i8 MFMA, or dense fp6 MFMA for the
        # fp6 screen (no sparsity in either)
        peak, unit = (FP6_MFMA_PEAK_TFLOPS if fp6 else I8_MFMA_PEAK_TOPS), "TFLOP/s"
        dom_ms = screen_ms if screened else kernel_ms
        achieved = alg_ops / (dom_ms * 1e-3) / 1e12
        if fp6:
            # tile pairs (two tiles sharing one A image per workgroup) from
            # WLD_OPT_FP6_PAIRS_MIN_TILES tiles (default 0) while the pair
            # list's 15-bit tile index holds the sites
            pairs_min = ctx.get_option("fp6_pairs_min_tiles")
            kname = ("pair_fp6_screen2w_kernel<tile pairs, 32x64 per wave, fp6 x fp4 16x16x128>"
                     if (L + 63) // 64 <= 0x7FFF and n_tiles >= pairs_min
                     else "pair_fp6_screen_kernel<fp6 x fp4 16x16x128>")
        elif screen_kind == 4:
            kname = "pair_mfma_kernel<candidate pairs, %d planes>" % min(planes, 2)
        elif screened and screen_kind == 1 and ctx.get_option("i8_pairs") and NP <= 16384 and \
                bool(np.all(weights >= 0)) and (L + 63) // 64 <= 0x7FFF:
            # the i8 one-plane screen on the tile-pair list (WLD_OPT_I8_PAIRS)
            kname = "pair_i8_screen2w_kernel<tile pairs, 32x64 per wave, i8 16x16x64, pre-multiplied operands>"
        elif screened:
            kname = "pair_mfma_kernel<screen,%d plane%s>" % ((2, "s") if screen_kind == 3 else (1, ""))
        else:
            kname = "pair_mfma_kernel<%d planes>" % planes
        roof = {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": unit, "frac": achieved / peak,
                "work": "algorithmic: 8*N ops per site pair (4 masked weighted sums)",
                "kernel": kname, "kernel_ms": dom_ms}
        # what the matrix cores executed: P digit planes x 8 N per pair (one
        # or two i8 planes when screened)
        ex_planes = (2 if screen_kind == 3 else 1) if screened and screen_kind != 4 else \
            min(planes, 2) if screen_kind == 4 else planes
        roof["executed_frac"] = shard_pairs * 8.0 * ex_planes * N / (dom_ms * 1e-3) / 1e12 / peak
        roof["executed_work"] = ("fp6 weights x fp4 codes, 8*N ops per pair" if fp6 else
                                 "%d i8 digit plane(s) x 8*N ops per pair" % ex_planes)
        # against the i8 peak as well (the integer kernels' roofline)
        roof["frac_of_i8_peak"] = achieved / I8_MFMA_PEAK_TOPS
    else:
        achieved = alg_ops / (kernel_ms * 1e-3) / 1e12
        # finite weights: f32-input MFMA (v_mfma_f32_16x16x4_f32), whose peak is the
        # f32 vector peak (MI355X_MICROARCH.md, Matrix cores: F32 row)
        roof = {"bound": "mfma", "achieved": achieved, "peak": F32_VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": achieved / F32_VALU_PEAK_TFLOPS, "path": "f32 MFMA 16x16x4",
                "work": "algorithmic: 8*N f32 flops per site pair",
                # (lib.rs's order on up to 4 x 768 tiles: 16-row items, one
                # sub-block per wave, capi.hip / pair_valu.hip ref_item_kernel)
                "kernel": ("ref_item_kernel<lib.rs order, 16-row items>" if args.ref_sums and n_tiles <= 4 * 768
                           else "pair_valu_kernel<%s>" % ("lib.rs order" if args.ref_sums else "two-level sums")),
                "kernel_ms": kernel_ms}
    roof["pair_phase_ms"] = kernel_ms
    roof["pair_phase_frac"] = alg_ops / (kernel_ms * 1e-3) / 1e12 / roof["peak"]
    if screened:
        n_cand = float(np.mean(cand))
        cand_ms = kernel_ms - screen_ms
        # the candidate launch: every plane of its tiles (or, --ref-sums, the
        # f32 reference-order kernel), algorithmic work 8N per pair of its
        # tiles (4096 pairs each, diagonal tiles counted whole)
        cand_peak = F32_VALU_PEAK_TFLOPS if args.ref_sums else I8_MFMA_PEAK_TOPS
        cand_ops = n_cand * 4096 * 8.0 * N
        if screen_kind == 4:  # the per-pair kernel's algorithmic work: 8N per candidate pair
            cand_ops = float(np.mean(cpairs)) * 8.0 * N
        roof["screen"] = {"kind": "fp6 x fp4" if fp6 else {3: "i8 two-plane", 4: "candidate pairs (i8 pass on the top two digit planes, rigorous bound)"}.get(screen_kind, "i8"),
                          "tiles": n_tiles,
                          "candidate_tiles": n_cand, "candidate_fraction": n_cand / max(n_tiles, 1),
                          "screen_ms": screen_ms, "candidate_launch_ms": cand_ms,
                          "candidate_kernel": ("ref_rows_kernel<lib.rs order, one pair per thread>" if screen_kind == 4
                                               else "ref_item_kernel<lib.rs order, f32 MFMA, 16-row items>" if args.ref_sums else
                                               "pair_mfma_kernel<prefilter, %d planes>" % planes),
                          "candidate_pairs": float(np.mean(cpairs)) if screen_kind == 4 else None,
                          "candidate_frac": (cand_ops / (cand_ms * 1e-3) / 1e12 / cand_peak) if cand_ms > 0.02 else None,
                          "candidate_peak": cand_peak,
                          # --ref-sums computes only the candidate tiles' 16x16
                          # sub-blocks holding a pair the screen could not reject
                          "candidate_blocks": float(np.mean(cblk)),
                          "candidate_computed_frac": ((float(np.mean(cblk)) * 256 * 8.0 * N) / (cand_ms * 1e-3) / 1e12
                                                      / cand_peak) if cand_ms > 0.02 and args.ref_sums else None,
                          "unscreened_pair_kernel_ms": unscreened_ms,
                          "unscreened_frac": alg_ops / (unscreened_ms * 1e-3) / 1e12 / roof["peak"]}
    # PMC traffic (profiles/traffic.json) was measured on the default C4 line's
    # dominant kernel (the one-plane i8 screen); other lines report null
    # (keyed by the data set too: the same kernel moves different bytes on linkage blocks)
    tr = load_traffic(args.config + ("-unweighted" if args.unweighted else "") +
                      ("-ldblocks" if args.data == "ldblocks" else ""),
                      "fp6" if fp6 else "i8pairs" if roof.get("kernel", "").startswith("pair_i8_screen2w") else kern_name)
    same_kernel = (screen_kind == 1 and args.thr is None and not args.wide_weights
                   and not (args.rehearse_dist and args.rehearse_shard > 1))
    # ... and only for the kernel those counters were collected on
    if tr and tr.get("kernel") and tr["kernel"].split("<")[0] != roof.get("kernel", "").split("<")[0]:
        tr = None
    roof["traffic"] = tr.get("hbm_bytes_per_launch") if tr and same_kernel else None
    hbm_alg = shard_pairs * 2.0 * N / (kernel_ms * 1e-3) / 1e9  # 2N bytes per pair
    # the arithmetic the timed steps executed
    fixed = "%d-bit fixed-point weights" % (31 if planes == 4 else 23)
    if kern_name == "mfma" and screen_kind == 4:
        dtype = ("i8 MFMA on the top %d digit plane(s) of %s (i32 sums), rigorous r2 bound with lib.rs's rounding; "
                 "the %.0f candidate pairs: f32 sums in lib.rs's order, f32 epilogue" % (
                     min(planes, 2), fixed, float(np.mean(cpairs))))
    elif kern_name == "mfma" and fp6:
        dtype = ("fp6 (e2m3) weights x fp4 (e2m1) codes on block-scaled MFMA, screen (f32 sums, exact on the rounded "
                 "weights; rigorous f32 r2 bound over every pair); candidate tiles (%.0f of %d): %s" % (
                     float(np.mean(cand)), n_tiles,
                     "f32 sums in lib.rs's order on f32 MFMA, f32 epilogue" if args.ref_sums else
                     "%d i8 digit plane%s of %s, exact i32 sums, f32 epilogue" % (planes, "s" if planes > 1 else "",
                                                                                  fixed)))
    elif kern_name == "mfma" and screened:
        dtype = ("i8 MFMA screen on the top weight digit%s (i32 sums, rigorous f32/f64 r2 bound over every pair); "
                 "candidate tiles (%.0f of %d): %s" % (
                     "s (2 planes)" if screen_kind == 3 else " (1 plane)", float(np.mean(cand)), n_tiles,
                     "f32 sums in lib.rs's order on f32 MFMA, f32 epilogue" if args.ref_sums else
                     "%d i8 digit plane%s of %s, exact i32 sums, f32 epilogue" % (planes, "s" if planes > 1 else "",
                                                                                  fixed)))
    elif kern_name == "mfma" and not args.ref_sums:
        dtype = "i8 MFMA, %d digit plane%s of %s, exact i32 sums, f32 epilogue" % (planes, "s" if planes > 1 else "",
                                                                                   fixed)
    else:
        dtype = "f32 MFMA (exact products, f32 sums%s), f32 epilogue" % (
            " in lib.rs's order" if args.ref_sums else "")
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "site-pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "settle_steps": settle_steps,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": dtype,
        "data": "synthetic (%s, %s weights)" % (
            "seeded bench_weighted_pair_ld.rs distribution" if args.data == "random" else
            "seeded linkage blocks of 20-200 sites (bench.ld_blocks)",
            "unit (--unweighted)" if args.unweighted else
            "Henikoff, every 10th x 2^-8 (--wide-weights)" if args.wide_weights else "Henikoff"),
        "config": {"workload": desc, "n_seqs": N, "n_sites": L, "r2_threshold": thr, "pairs": total_pairs,
                   "rows_passing": rows, "kernel": kern_name, "mfma_planes": planes,
                   "library_options": os.environ.get("WLD_BENCH_OPTS") or "defaults",
                   "launch": ("bench.py spawned %d ranks" % world if os.environ.get("WLD_BENCH_SPAWNED") else
                              "external launcher (WORLD_SIZE=%d)" % world if "WORLD_SIZE" in os.environ else
                              "single process"),
                   # gloo host collectives may put several ranks on one GPU
                   # (the launcher's multi-rank test): count the devices used
                   "devices": min(world, n_dev) if host_coll else world,
                   "parallelism": "chunk-range shard x%d%s%s" % (
                       world, (((" + row counts through host shared memory" if xchg is not None else
                                 " + gloo host-tensor count all_gather" if host_coll else " + RCCL count all_gather") +
                                (", gloo host-tensor row gather" if host_coll else ", exact-size RCCL send/recv of the "
                                 "rows to rank 0")) if dist_on else ""),
                       (", pipelined steps (%d contexts, %s)" % (
                           depth, {"0": "screens may overlap", "1": "serialized on the whole step",
                                   "stream": "one stream"}.get(
                               serialize, "pair kernels queued back to back") +
                           (" (auto: the faster of two interleaved trials of each order)"
                            if serialize_trials else ""))
                        if (pipe is not None or ctxs1 is not None) else ""))},
        "roofline": roof,
        # N=1 "auto": ms/step of each trial of the two step orders (the timed steps ran the faster)
        "pipe_order_trials_ms": serialize_trials,
        # SURVEY 8(d)'s no-reuse byte MODEL (2N bytes per pair as if every pair
        # re-read both site columns from HBM) — not a roofline: the kernel
        # stages columns through LDS/L2 and reads each far fewer times
        "north_star_hbm_model": {"model_bytes_per_pair": 2 * N, "model_GBps": hbm_alg,
                                 "hbm_peak_GBps": HBM_PEAK_GBPS, "model_over_peak": hbm_alg / HBM_PEAK_GBPS},
        "order_ms": float(np.mean(oms)),
        # SURVEY 8(d) timing window: phases outside `value`'s step are reported, not timed in it
        "phases_ms": {"host_prepass_filter_henikoff": prepass_ms,
                      "device_prepass_filter_henikoff_encode": float(min(dev_ms)), "h2d_inputs": h2d_ms,
                      "device_encode_prep": load_ms, "pair_phase": kernel_ms, "order_assembly": float(np.mean(oms)),
                      "step_minus_kernel_rank0": float(np.median(gms))},
    }
    if checked:
        # every checked step's rows (gathered to rank 0 at N>1) against the
        # oracle over the same chunk range: the same rows in the same order,
        # d / d' / r2 bit for bit in lib.rs's order (within 1e-5 otherwise)
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import _oracle as O  # checker only
        O.use_native()
        ref = O.all_pairs(buf, weights, np.float32(thr), n_threads=int(os.environ.get("OMP_NUM_THREADS") or 0) or
                          (os.cpu_count() or 1), chunk_lo=0 if world > 1 else cb, chunk_hi=ctx.chunks(L)
                          if world > 1 else ce)
        equal = 0
        for g in checked:
            same = len(g["site_a"]) == len(ref["site_a"]) and all(
                np.array_equal(g[f].astype(np.uint32), ref[f].astype(np.uint32)) for f in ("site_a", "site_b"))
            for f in ("d", "d_prime", "r2"):
                if not same:
                    break
                a, b = np.asarray(g[f], dtype=np.float32), np.asarray(ref[f], dtype=np.float32)
                same = np.array_equal(a.view(np.uint32), b.view(np.uint32)) if args.ref_sums else bool(
                    np.all(np.abs(a.astype(np.float64) - b) <= 1e-5 * np.maximum(1.0, np.abs(b))))
            equal += bool(same)
        out["steps_check"] = {"steps": len(checked), "equal_to_oracle": equal, "rows_per_step": len(ref["site_a"]),
                              "compare": "bitwise" if args.ref_sums else "within 1e-5"}
        assert equal == len(checked) == args.check_steps, out["steps_check"]
    if args.no_cpu_baseline:
        out["cpu_baseline"] = None
    else:
        # rank 0 (at N>1 after the other ranks have left: no rank polls beside
        # it), a bounded sample at N>1 so that a scaling run stays short
        oref, ochunks, out["cpu_baseline"] = cpu_baseline(buf, weights, thr, args.cpu_seconds if world == 1 else
                                                          min(args.cpu_seconds, 5.0),
                                                          max_s=30.0 if world == 1 else 8.0)
        # the same chunks on the GPU: rows against the oracle's (lib.rs
        # semantics).  Exact sums rounded once may put a pair whose r2 lies
        # within 1e-5 of the threshold on the other side of the strict '>'
        # (never more); --ref-sums must match exactly.
        ctx.run_chunks(thr, 0, ochunks)
        g = ctx.rows()
        kg = set(zip(g.site_a.tolist(), g.site_b.tolist()))
        kr = set(zip(oref["site_a"].tolist(), oref["site_b"].tolist()))
        r2g = dict(zip(zip(g.site_a.tolist(), g.site_b.tolist()), g.r2.tolist()))
        r2r = dict(zip(zip(oref["site_a"].tolist(), oref["site_b"].tolist()), oref["r2"].tolist()))
        one_sided = [r2g[k] for k in kg - kr] + [r2r[k] for k in kr - kg]
        out["rows_check"] = {"chunks": ochunks, "gpu_rows": len(kg), "oracle_rows": len(kr),
                             "one_sided": len(one_sided),
                             "one_sided_outside_1e-5_of_thr": sum(abs(v - thr) > 1e-5 for v in one_sided)}
        whole = ochunks == ctx.chunks(L) and (cb, ce) == (0, ctx.chunks(L))
        if whole:
            out["rows_check"]["timed_rows_passing"] = rows  # the last timed step's rows: the same run
        assert out["rows_check"]["one_sided_outside_1e-5_of_thr"] == 0, out["rows_check"]
        assert not args.ref_sums or len(one_sided) == 0, out["rows_check"]
        assert not whole or rows == len(kg), (rows, len(kg))
        if fp6 and whole and world == 1 and len(kr) < 1000 and args.ref_sums and args.config == "c4":
            # the check above is vacuous where no row passes (C4 at 0.05): the
            # same size and threshold with planted linkage, the fp6 screen
            # forced and auto, every row against the oracle (rows, order, bits)
            out["rows_check_fp6"] = fp6_planted_check(W, dev_index, L, N, thr)
            assert out["rows_check_fp6"]["equal"], out["rows_check_fp6"]
    print(json.dumps(out), flush=True)
    close_all()


if __name__ == "__main__":
    main()
