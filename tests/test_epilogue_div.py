"""The epilogue's eight quotients by the total weight (pair_common.hpp
ld_epilogue, WLD_EPI_DIVT): RN_f32(x * r) in f64 with a Newton-refined
reciprocal must be the IEEE f32 quotient x / T (lib.rs:491-502 divides each in
f32) for every input — checked on the host from a coarser starting estimate
than the device's (tests/cpp/div_check.cpp).  The GPU parity tests then check
the device's rows and stats bit for bit against the oracle."""
import os
import subprocess

from conftest import REPO


def test_quotients_equal_ieee_division(tmp_path):
    exe = str(tmp_path / "div_check")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17", "-ffp-contract=off",
                    "-I", os.path.join(REPO, "include"), "-I", os.path.join(REPO, "weightedld_amd", "csrc"),
                    "-x", "hip", os.path.join(REPO, "tests", "cpp", "div_check.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe, "6000000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout
