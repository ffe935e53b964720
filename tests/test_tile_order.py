"""The run tile lists (weightedld_amd/csrc/tile_order.hpp, capi.hip
build_tiles) equal the round-4 sort-based builder, element for element, for
whole sets and shards (tests/cpp/tile_order_check.cpp, host only)."""
import os
import subprocess

from conftest import REPO


def test_tile_lists_equal_sort_based_builder(tmp_path):
    exe = str(tmp_path / "tile_order_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(REPO, "weightedld_amd", "csrc"),
                    os.path.join(REPO, "tests", "cpp", "tile_order_check.cpp"), "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.strip().endswith("OK"), out.stdout + out.stderr
