// Where each 64x64 tile of a whole-set run sits in the fp6 screen's launch
// (capi.hip build_tiles: tile_order.hpp range_tiles -> fp6_pair_list ->
// xcd_order): one line per tile "ta tb xcd kind", xcd = the XCD queue of its
// entry (launch position mod 8), kind 0 / 1 = first / second half of a tile
// pair, 2 = a single entry.  Host only (tests/test_planted.py).
//   f6_entry_map L NP
#include <cstdio>
#include <cstdlib>
#include "tile_order.hpp"

using namespace wld::tile_order;

int main(int argc, char **argv) {
    if (argc != 3) return 2;
    const uint32_t L = (uint32_t)atoi(argv[1]), NP = (uint32_t)atoi(argv[2]);
    const uint32_t T_used = (L + 63) / 64, n = (L + 255) / 256;
    const uint32_t nchunks = n * (n + 1) / 2;
    const std::vector<uint32_t> t = range_tiles(n, T_used, 0, nchunks);
    std::vector<uint32_t> pl = fp6_pair_list(t);
    if (pl.size() >= 2048) pl = xcd_order(pl, super_block_side(NP), ~kSingleEntry);
    for (size_t i = 0; i < pl.size(); ++i) {
        const uint32_t e = pl[i];
        if (e == kNoTileEntry) continue;
        const uint32_t ta = e >> 16, tb = e & 0x7FFFu;
        if (e & kSingleEntry) {
            printf("%u %u %zu 2\n", ta, tb, i % 8);
        } else {
            printf("%u %u %zu 0\n", ta, tb, i % 8);
            printf("%u %u %zu 1\n", ta, tb + 1, i % 8);
        }
    }
    return 0;
}
