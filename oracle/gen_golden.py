#!/usr/bin/env python3
"""Generate the committed golden vectors under tests/golden/ from the Python reference.

TEST INFRASTRUCTURE ONLY — never imported by the product path, bench.py's GPU leg
or anything that runs on the GPU box.  It needs /root/reference (this container
only) and writes small JSON/FASTA fixtures that travel instead.

What it does
------------
* Writes seeded synthetic alignments (tests/golden/synthetic/*.fasta) drawn with
  the distribution of the reference microbench generator
  (rust/weighted_ld/benches/bench_weighted_pair_ld.rs:8-28: 10% '-', 60% major,
  rest minor; here seeded, not thread_rng).
* Imports /root/reference/WeightedLD.py in a child interpreter with the four
  harness-only shims of SURVEY.md Appendix C (a tiny Bio.AlignIO FASTA reader,
  np.bool8, a numpy-1 style uint8 cast for handle_vcf, and an un-rounding
  `round` so D/D'/r2 come out at full f64 precision while the `round(PA, 1)` skip
  rule of WeightedLD.py:234-237 is left intact).
* Records, per case: the variable-site masks (WeightedLD.py:44-98), Henikoff
  weights (:101-151) and every `ld()` row (:154-284), unrounded.
* Records the lib.rs unit-test known answers (lib.rs:691-801) as data.

Run:  python3 oracle/gen_golden.py        (from the repo root, in this container)
"""
import json
import os
import subprocess
import sys
import tempfile
import textwrap

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
GOLDEN = os.path.join(REPO, "tests", "golden")
FIXTURES = os.path.join(GOLDEN, "fixtures")
SYNTH = os.path.join(GOLDEN, "synthetic")

FASTA_CASES = [
    "example.fasta",
    "t1_henikoff_paper.fasta",
    "t2_henikoff_complex1.fasta",
    "t3_henikoff_complex2.fasta",
    "t4_weights1_ld0.fasta",
    "t5_weights1_ld0.25.fasta",
    "t6_varsites_hk_ld.fasta",
]

# (name, n_seqs, n_sites, seed)
SYNTH_CASES = [
    ("synth_n200_l24", 200, 24, 11),
    ("synth_n500_l40", 500, 40, 12),
    ("synth_n2000_l30", 2000, 30, 13),
]

SYMS = "ACGT-"


def write_synthetic(path, n_seqs, n_sites, seed):
    """Seeded version of bench_weighted_pair_ld.rs:8-28 (per site: major != minor
    drawn from ACGT; each sequence '-' w.p. 0.10, major w.p. 0.60, else minor).
    One sequence per line with a trailing newline (lib.rs:277-307 reads lines)."""
    import numpy as np

    rng = np.random.Generator(np.random.PCG64(seed))
    maj = rng.integers(0, 4, size=n_sites)
    off = rng.integers(1, 4, size=n_sites)
    mnr = (maj + off) % 4
    u = rng.random((n_seqs, n_sites))
    codes = np.where(u < 0.10, 4, np.where(u < 0.70, maj[None, :], mnr[None, :]))
    table = np.frombuffer(SYMS.encode(), dtype=np.uint8)
    chars = table[codes]
    with open(path, "w") as f:
        for i in range(n_seqs):
            f.write(">s%d\n" % i)
            f.write(chars[i].tobytes().decode() + "\n")


SHIM_ALIGNIO = '''
class _Rec:
    def __init__(self, name, seq):
        self.id = name
        self.seq = seq

class _Aln(list):
    def get_alignment_length(self):
        return len(self[0].seq)

def read(filename, fmt):
    assert fmt == "fasta"
    recs, name, buf = [], None, []
    with open(filename) as f:
        for line in f:
            line = line.strip()
            if line.startswith(">"):
                if name is not None:
                    recs.append(_Rec(name, "".join(buf)))
                name, buf = line[1:], []
            elif line:
                buf.append(line)
    if name is not None:
        recs.append(_Rec(name, "".join(buf)))
    n = len(recs[0].seq)
    if any(len(r.seq) != n for r in recs):
        raise ValueError("Sequences must all be the same length")
    return _Aln(recs)
'''

SHIM_SITECUSTOMIZE = '''
import numpy as np
if not hasattr(np, "bool8"):
    np.bool8 = np.bool_
'''

CHILD = r'''
import builtins, contextlib, io, json, sys, types
import numpy as np
sys.path.insert(0, "/root/reference")
import WeightedLD as wld

# shim 4: unrounded outputs, keep round(PA, 1) (WeightedLD.py:234-237)
wld.round = lambda x, nd=None: x if nd == 4 else builtins.round(x, nd)

# shim 3: numpy-1 style list -> uint8 cast used by handle_vcf (WeightedLD.py:372)
proxy = types.ModuleType("np_proxy")
proxy.__dict__.update(np.__dict__)
def _array(o, dtype=None, **k):
    if dtype is np.uint8 and isinstance(o, list):
        return np.array(o, dtype=np.int64).astype(np.uint8)
    return np.array(o, dtype=dtype, **k)
proxy.array = _array
wld.np = proxy

def run_ld(alignment, weights, site_map):
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        wld.ld(alignment, weights, site_map)
    lines = buf.getvalue().splitlines()
    assert lines[0] == "posa\tposb\tD\tD'\tR2", lines[0]
    rows = []
    for ln in lines[1:]:
        a, b, d, dp, r2 = ln.split("\t")
        rows.append([int(a), int(b), float(d), float(dp), float(r2)])
    return rows

def fasta_case(path, min_acgt=0.8, min_var=0.02):
    aln = wld.read_fasta(path)
    hk, ldm = wld.compute_variable_sites(aln, min_acgt, min_var)
    out = {"n_seqs": int(aln.shape[0]), "n_sites": int(aln.shape[1]),
           "alignment_sum": int(aln.sum()),
           "var_sites_hk": [bool(x) for x in hk], "var_sites_ld": [bool(x) for x in ldm]}
    sub = aln[:, ldm]
    site_map = np.where(ldm)[0]
    if sub.shape[1] > 0:
        w = wld.henikoff_weighting(sub)
        out["weights"] = [float(x) for x in w]
        out["pairs_weighted"] = run_ld(sub, w, site_map)
    else:
        out["weights"] = []
        out["pairs_weighted"] = []
    uw = np.zeros(sub.shape[0], dtype=np.uint8); uw[uw == 0] = 1
    out["pairs_unweighted"] = run_ld(sub, uw, site_map) if sub.shape[1] > 0 else []
    # Henikoff on the HK mask (test.py:37-67 style)
    hks = aln[:, hk]
    out["weights_hk_sites"] = [float(x) for x in wld.henikoff_weighting(hks)] if hks.shape[1] else []
    return out

def vcf_case(path):
    aln, site_map = wld.handle_vcf(path)
    w = wld.henikoff_weighting(aln)
    uw = np.zeros(aln.shape[0], dtype=np.uint8); uw[uw == 0] = 1
    return {"n_seqs": int(aln.shape[0]), "n_sites": int(aln.shape[1]),
            "site_map": [int(x) for x in site_map],
            "weights_mean": float(w.mean()),
            "weights": [float(x) for x in w],
            "alignment_T": ["".join(str(int(v)) for v in col) for col in aln.T],
            "pairs_weighted": run_ld(aln, w, site_map),
            "pairs_unweighted": run_ld(aln, uw, site_map)}

req = json.loads(sys.stdin.read())
res = {}
for name, path in req["fasta"]:
    res[name] = fasta_case(path)
for name, path in req["vcf"]:
    res[name] = vcf_case(path)
# test.py:69-101 variants (different filter parameters)
res["t4_weights1_ld0.fasta@0.99"] = fasta_case(req["t4"], 0.99, 0.02)
res["t4_weights1_ld0.fasta@0.1,0.2"] = fasta_case(req["t4"], 0.1, 0.2)
res["t6_varsites_hk_ld.fasta@0.8,0.2"] = fasta_case(req["t6"], 0.8, 0.2)
json.dump(res, sys.stdout)
'''

LIBRS_KNOWN_ANSWERS = {
    "_source": "rust/weighted_ld/src/lib.rs:686-802 (#[cfg(test)] mod tests) — inputs and expected values as data",
    "histogram": {"ref": "lib.rs:691-703", "symbols": "AAACCGTTTT--N", "expect": [3, 2, 1, 4, 2, 1]},
    "major_minor": {"ref": "lib.rs:704-728", "cases": [
        {"hist": [0, 1, 10, 2, 0, 0], "major": 2, "minor": 3},
        {"hist": [1, 9, 10, 2, 0, 0], "major": 2, "minor": 1},
        {"hist": [1, 1, 40, 2, 4, 0], "major": 2, "minor": 4}]},
    "henikoff": {"cases": [
        {"ref": "lib.rs:730-735", "seqs": ["AAAAA", "AAAAA", "CCCCC", "CCCCC", "TTTTT"],
         "expect": [0.5, 0.5, 0.5, 0.5, 1.0], "tol": "ulps"},
        {"ref": "lib.rs:737-742", "seqs": ["GCGTTAGC", "GAGTTGGA", "CGGACTAA"],
         "expect": [0.769, 0.692, 1.0], "tol": 1e-3},
        {"ref": "lib.rs:744-750", "seqs": ["AAGA", "AA-A", "GGGG", "GGGG"],
         "expect": [0.733, 1.0, 0.733, 0.733], "tol": 1e-3}]},
    "ld_pair": {"cases": [
        {"ref": "lib.rs:752-767", "a": "AAAATTTT", "b": "TTAAAATT", "w": [1.0] * 8,
         "d": 0.0, "d_prime": 0.0, "r2": 0.0, "tol": 1e-5},
        {"ref": "lib.rs:769-784", "a": "AAAATTTT", "b": "TTTTAAAA", "w": [1.0] * 8,
         "d": 0.25, "d_prime": 0.5, "r2": 1.0, "tol": 1e-5},
        {"ref": "lib.rs:786-801", "a": "AAAACAC", "b": "AAAGTAA",
         "w": [1.0, 1.0, 0.4, 0.2, 0.5, 0.8, 0.2],
         "d": 0.00308, "d_prime": 0.05555, "r2": 0.00346, "tol": 1e-5}]},
}


def main():
    os.makedirs(SYNTH, exist_ok=True)
    synth_paths = []
    for name, n, l, seed in SYNTH_CASES:
        p = os.path.join(SYNTH, name + ".fasta")
        write_synthetic(p, n, l, seed)
        synth_paths.append((name + ".fasta", p))

    req = {
        "fasta": [(c, os.path.join(FIXTURES, c)) for c in FASTA_CASES] + synth_paths,
        "vcf": [("t7_1000genome.vcf", os.path.join(FIXTURES, "t7_1000genome.vcf"))],
        "t4": os.path.join(FIXTURES, "t4_weights1_ld0.fasta"),
        "t6": os.path.join(FIXTURES, "t6_varsites_hk_ld.fasta"),
    }
    with tempfile.TemporaryDirectory() as shim:
        os.makedirs(os.path.join(shim, "Bio"))
        open(os.path.join(shim, "Bio", "__init__.py"), "w").close()
        with open(os.path.join(shim, "Bio", "AlignIO.py"), "w") as f:
            f.write(textwrap.dedent(SHIM_ALIGNIO))
        with open(os.path.join(shim, "sitecustomize.py"), "w") as f:
            f.write(textwrap.dedent(SHIM_SITECUSTOMIZE))
        env = dict(os.environ, PYTHONPATH=shim, PYTHONDONTWRITEBYTECODE="1")
        proc = subprocess.run([sys.executable, "-c", CHILD], input=json.dumps(req),
                              capture_output=True, text=True, env=env, cwd=REF)
        if proc.returncode != 0:
            sys.stderr.write(proc.stderr)
            raise SystemExit("python reference run failed")
        res = json.loads(proc.stdout)

    meta = {
        "_source": "WeightedLD.py (reference Python implementation) run under the harness shims of "
                   "SURVEY.md Appendix C by oracle/gen_golden.py; values unrounded (f64).",
        "_synthetic": {name + ".fasta": {"n_seqs": n, "n_sites": l, "seed": seed}
                       for name, n, l, seed in SYNTH_CASES},
    }
    out = {"meta": meta, "cases": res}
    with open(os.path.join(GOLDEN, "python_ref.json"), "w") as f:
        json.dump(out, f, sort_keys=True, separators=(",", ":"))
    with open(os.path.join(GOLDEN, "librs_known_answers.json"), "w") as f:
        json.dump(LIBRS_KNOWN_ANSWERS, f, indent=1, sort_keys=True)
    for k, v in res.items():
        print("%-36s seqs=%-5d sites=%-3d weighted=%-4d unweighted=%d" % (
            k, v["n_seqs"], v["n_sites"], len(v["pairs_weighted"]), len(v["pairs_unweighted"])))


if __name__ == "__main__":
    main()
