"""bench.py's contract: the synthetic inputs (CPU) and the one JSON line a
short default run prints (GPU, run as a child process exactly as the driver
runs it)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_synth_distribution_and_seed():
    """bench_weighted_pair_ld.rs:8-28's distribution: '-' 0.10, major 0.60,
    minor 0.30, per site a major != minor from ACGT; seeded."""
    a = bench.synth(300, 2000)
    assert a.shape == (300, 2000) and a.dtype == np.uint8
    assert np.array_equal(a, bench.synth(300, 2000))
    gap = (a == 4).mean()
    assert abs(gap - 0.10) < 0.005
    for s in range(0, 300, 37):
        row = a[s][a[s] != 4]
        vals, cnt = np.unique(row, return_counts=True)
        assert len(vals) == 2 and vals.max() < 4
        assert abs(cnt.max() / len(row) - 2 / 3) < 0.05  # major 0.6 of 0.9


def test_ld_blocks_and_vcf_like_shapes():
    b = bench.ld_blocks(500, 300)
    assert b.shape == (500, 300) and np.array_equal(b, bench.ld_blocks(500, 300))
    assert set(np.unique(b)) <= {0, 1, 2, 3, 4}
    v = bench.vcf_like(200, n_hap=64)
    assert v.shape == (200, 64) and set(np.unique(v)) <= {0, 1, 4}


def test_pairs_in_rows_partition():
    """Row-block pair counts add up to L(L-1)/2 (the shard balance uses them)."""
    L = 20000
    blocks = (L + 255) // 256
    total = sum(bench.pairs_in_rows(L, r, r + 1) for r in range(blocks))
    assert total == L * (L - 1) // 2
    assert bench.pairs_in_rows(L, 0, blocks) == total


REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"}


@pytest.mark.gpu
def test_bench_json_line():
    """A short default-config run: one JSON line with the driver's keys, the
    roofline object, rows equal to the oracle's (bench asserts it)."""
    env = dict(os.environ)
    r = subprocess.run([sys.executable, "bench.py", "--steps", "5", "--warmup", "2", "--cpu-seconds", "2"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    assert REQUIRED <= set(out), sorted(REQUIRED - set(out))
    assert out["metric"] == bench.METRIC and out["n_gpus"] == 1 and out["steps"] == 5 and out["warmup"] == 2
    assert out["higher_is_better"] is True and out["value"] > 0 and out["ms_per_step"] > 0
    n_pairs = 20000 * 19999 // 2
    assert abs(out["value"] * out["ms_per_step"] / 1e3 / n_pairs - 1) < 0.01
    rf = out["roofline"]
    assert {"bound", "achieved", "peak", "unit", "frac", "traffic"} <= set(rf)
    assert 0 < rf["frac"] < 1 and abs(rf["achieved"] / rf["peak"] - rf["frac"]) < 1e-3
    cb = out["cpu_baseline"]
    assert cb["kind"] in ("port", "reference") and cb["value"] > 0 and cb["cores"] >= 1
    assert out["config"]["workload"]
    # N=1 auto step order: two trials of each order, the timed steps in the faster
    tr = out["pipe_order_trials_ms"]
    assert set(tr) == {"pair", "0"} and all(len(v) == 2 and min(v) > 0 for v in tr.values())
    chosen = "screens may overlap" if sum(tr["0"]) < sum(tr["pair"]) else "pair kernels queued back to back"
    assert chosen in out["config"]["parallelism"], out["config"]["parallelism"]


def test_launcher_starts_n_ranks_before_the_gpu():
    """--gpus 2 with no WORLD_SIZE: bench.py starts ranks 0 and 1 itself
    (RANK/LOCAL_RANK/WORLD_SIZE set, no external launcher); here, with no GPU,
    each rank stops with its own error and the launcher returns nonzero with
    no JSON line on stdout."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""  # (a GPU box too: no device for the ranks)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert "rank 0 of 2" in r.stderr + r.stdout or "rank 1 of 2" in r.stderr + r.stdout, r.stderr[-2000:]


def test_world_size_must_match_gpus():
    """Under an external launcher WORLD_SIZE must equal --gpus (no silent
    fallback to another rank count)."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--steps", "1"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "--gpus 4 but WORLD_SIZE=2" in r.stderr


@pytest.mark.gpu
def test_launcher_two_ranks_rows_equal_oracle_every_step():
    """`bench.py --gpus 2` starts its own two ranks (here both on the box's one
    GPU, counts and rows exchanged as host tensors over gloo); BASELINE config
    2 at threshold 0 (1,999,000 rows a step, split over the two shards and
    gathered to rank 0 with exact-size transfers): every checked step's rows
    equal the oracle's bit for bit, in reference order; the line says n_gpus 2
    and leaves the CPU baseline (an N=1 figure) null."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--collectives", "gloo", "--config", "c2",
                        "--steps", "5", "--warmup", "2", "--settle-s", "0", "--check-steps", "4",
                        "--cpu-seconds", "2", "--counts", "collective"], cwd=REPO, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    assert REQUIRED <= set(out), sorted(REQUIRED - set(out))
    assert out["n_gpus"] == 2 and out["config"]["launch"] == "bench.py spawned 2 ranks"
    sc = out["steps_check"]
    assert sc["steps"] == 4 and sc["equal_to_oracle"] == 4 and sc["rows_per_step"] > 1_900_000
    assert out["config"]["rows_passing"] == sc["rows_per_step"]
    # an N>1 line carries rank 0's CPU baseline too (after the other ranks left),
    # on the CPUs the process may use, the count justified in the record
    cb = out["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1
    assert cb["host_cpus"]["affinity"] >= cb["cores"] and cb["host_cpus"]["threads_from"]
    assert out["rows_check"]["one_sided"] == 0


@pytest.mark.gpu
def test_launcher_eight_ranks_rows_equal_oracle_every_step():
    """the driver's N=8 launch path, run once before its SCALE
    run does: `bench.py --gpus 8` spawns eight ranks (here all on the box's
    one GPU, counts and rows over gloo host tensors: a functional check, not a
    performance line); BASELINE config 2 at threshold 0, each rank's 1/8
    chunk range, the pipelined N>1 step loop; both checked steps' gathered
    rows equal the oracle's bit for bit in reference order, and the line says
    n_gpus 8.  The row counts go through host shared memory (--counts auto on
    one host; the two-rank test above keeps the collective count exchange)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--collectives", "gloo", "--config", "c2",
                        "--steps", "3", "--warmup", "1", "--settle-s", "0", "--check-steps", "2",
                        "--cpu-seconds", "1"], cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["config"]["launch"] == "bench.py spawned 8 ranks"
    assert "host shared memory" in out["config"]["parallelism"], out["config"]
    sc = out["steps_check"]
    assert sc["steps"] == 2 and sc["equal_to_oracle"] == 2 and sc["rows_per_step"] > 1_900_000
    print("eight ranks: %.3f ms/step (one shared GPU), steps_check %s" % (out["ms_per_step"], sc))
