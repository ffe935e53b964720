"""The planted-linkage workload (bench.planted_ld) covers what VERDICT r5 #1
asks of the headline screen's full-size test, checked on the host: at
BASELINE config 4's size and threshold, >= 500 planted pairs pass (their r2
from the oracle's single_weighted_ld_pair, lib.rs:390-521) and the tiles
holding them (>= 300) fall on every XCD queue of the fp6 screen's launch, in
both halves of tile-pair entries and in single entries, on diagonal tiles and
in the padded last tile row and column (tests/cpp/f6_entry_map.cpp: the
launch list capi.hip builds, from tile_order.hpp)."""
import os
import subprocess

import numpy as np

import _oracle as O
from conftest import REPO


def test_planted_ld_covers_the_screen_launch(tmp_path):
    import sys
    sys.path.insert(0, REPO)
    import bench
    N, L, thr, _ = bench.CONFIGS["c4"]
    buf, planted = bench.planted_ld(L, N)
    assert buf.shape == (L, N)
    sites = [s for a, b, _ in planted for s in (a, b)]
    assert len(sites) == len(set(sites))  # every planted site used once
    w = O.henikoff_weights(buf)
    passing = []
    for a, b, _ in planted:
        _, _, r2 = O.single_pair(buf[a], buf[b], w)
        if np.float32(r2) > np.float32(thr):
            passing.append((a, b))
    tiles = {(a // 64, b // 64) for a, b in passing}
    assert len(passing) >= 500 and len(tiles) >= 300, (len(passing), len(tiles))
    assert len(passing) < len(planted)  # some planted pairs just below the threshold
    exe = str(tmp_path / "f6_entry_map")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(REPO, "weightedld_amd", "csrc"),
                    os.path.join(REPO, "tests", "cpp", "f6_entry_map.cpp"), "-o", exe], check=True)
    NP = -(-N // 64) * 64
    out = subprocess.run([exe, str(L), str(NP)], capture_output=True, text=True, check=True).stdout
    where = {}
    for line in out.splitlines():
        ta, tb, x, k = map(int, line.split())
        where[(ta, tb)] = (x, k)
    T = (L + 63) // 64
    assert len(where) == T * (T + 1) // 2
    xcd = {where[t][0] for t in tiles}
    kinds = {}
    for t in tiles:
        kinds[where[t][1]] = kinds.get(where[t][1], 0) + 1
    assert xcd == set(range(8)), xcd
    assert min(kinds.get(k, 0) for k in (0, 1, 2)) >= 10, kinds
    assert sum(a == b for a, b in tiles) >= 20
    assert (T - 1, T - 1) in tiles and sum(b == T - 1 for _, b in tiles) >= 10
    assert any(a % 2 == 1 and a == b for a, b in tiles) and any(a % 2 == 0 and a == b for a, b in tiles)
