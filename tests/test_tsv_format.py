"""TSV field formatting of the CLI writer (main.rs:76,82-119).

wld_tsv::fmt3 (weightedld_amd/csrc/tsv_format.hpp) prints Rust `{:.3}` of an
f32 with integer arithmetic instead of snprintf.  The checker program compares
it with glibc's "%.3f" of the widened double (exact binary value, ties to
even, as Rust's flt2dec format_exact).  All 2^32 bit patterns were checked
once with `tsv_format_check range` (0 mismatches); this test re-runs the edge
set, a random sample and every pattern of the exponent range [0.5, 1).
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("tsv") / "tsv_format_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "weightedld_amd", "csrc"), "-o", exe,
                    os.path.join(ROOT, "tests", "cpp", "tsv_format_check.cpp")], check=True)
    return exe


def _run(exe, *args):
    r = subprocess.run([exe, *args], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches=0" in r.stdout


def test_fmt3_sample(checker):
    _run(checker, "sample", "1000000", "11")


def test_fmt3_exponent_range_half_to_one(checker):
    # 0x3f000000 = 0.5f, 0x3f800000 = 1.0f: 2^23 patterns, both signs
    _run(checker, "range", "0x3f000000", "0x3f800000")
    _run(checker, "range", "0xbf000000", "0xbf800000")


def test_pipelined_writer_matches_serial(tmp_path):
    """write_pair_stats (cli.cpp) against a serial snprintf writer, byte for byte,
    at row counts around the 65536-row block size and one multi-block file."""
    exe = str(tmp_path / "tsv_writer_check")
    lib = os.path.join(ROOT, "weightedld_amd")
    if not os.path.exists(os.path.join(lib, "libweightedld.so")):
        pytest.skip("libweightedld.so not built")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-I",
                    os.path.join(lib, "csrc"), "-o", exe, os.path.join(ROOT, "tests", "cpp", "tsv_writer_check.cpp"),
                    "-L" + lib, "-lweightedld", "-Wl,-rpath," + lib, "-lpthread"], check=True)
    for n in (0, 1, 65535, 65536, 65537, 1000003):
        r = subprocess.run([exe, str(n), str(tmp_path)], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0 and "identical=1" in r.stdout, (n, r.stdout, r.stderr)
