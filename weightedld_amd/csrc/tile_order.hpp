// Host-side tile lists of a run (capi.hip build_tiles): the 64x64 tiles of a
// contiguous run of the reference's chunk sequence in (ta, tb) order, and the
// XCD-aware launch order of a tile (or tile-pair) list.  Header-only so the
// host test (tests/cpp/tile_order_check.cpp) checks the same code.
#pragma once
#include <algorithm>
#include <cstdint>
#include <vector>

namespace wld {
namespace tile_order {

constexpr uint32_t kNoTileEntry = 0xFFFFFFFFu;  // (= kernels.hpp kNoTile)

// Linear index of chunk (row, col) in the reference's triu_index order
// (lib.rs:623-632): rows descend, so row r starts at (n-1-r)(n-r)/2.
inline uint32_t chunk_linear_host(uint32_t n, uint32_t row, uint32_t col) {
    const uint32_t rf = n - 1 - row;
    return rf * (rf + 1) / 2 + (col - row);
}

// The tiles (tb >= ta, packed ta << 16 | tb) of the linear chunks [lb, le) of
// an n-chunk-row set with T_used tile rows (4 tiles per chunk side), in
// (ta, tb) order directly (no sort): row by row, the chunk columns in range.
inline std::vector<uint32_t> range_tiles(uint32_t n, uint32_t T_used, uint32_t lb, uint32_t le) {
    constexpr uint32_t kTilesPerChunkSide = 4;
    std::vector<uint32_t> t;
    for (uint32_t ta = 0; ta < T_used; ++ta) {
        const uint32_t row = ta / kTilesPerChunkSide;
        for (uint32_t col = row; col < n; ++col) {
            const uint32_t li = chunk_linear_host(n, row, col);
            if (li < lb || li >= le) continue;
            for (uint32_t tb = std::max(ta, col * kTilesPerChunkSide);
                 tb < std::min<uint32_t>((col + 1) * kTilesPerChunkSide, T_used); ++tb)
                t.push_back((ta << 16) | tb);
        }
    }
    return t;
}

// L2-aware launch order (default; WLD_TILE_ORDER=rows keeps plain (ta, tb)
// order): workgroups are dealt to the 8
// XCDs round-robin by launch index, so position 8i + x is XCD x's i-th tile.
// Each XCD gets whole kS x kS-tile super-blocks (greedy, least-loaded first),
// taken row by row; then the queues are evened out to within one tile.  Short
// queues are padded with kNoTileEntry entries, which the pair kernels skip.
// kS = 16 where the 128 screen tiles resident on an XCD's 32 CUs (4
// workgroups per CU: 8 rows of one super-block, 8 A and 16 B tile columns of
// 64 NP bytes) fit its 4 MB L2 (C4: 3 MB): 0.86 GB per C4 screen launch past
// L2 instead of 1.11 GB with kS = 8, step -0.5% (archive/profiles_r01_r03/r03ar, r03as,
// r03au).  Otherwise kS = 8, two whole super-blocks resident (C5, 323 KB
// columns: 3% faster than 16).
// The super-blocks in row-major block order, tiles inside a block ascending:
// a counting sort by block over the (ta, tb)-sorted list, O(n) (a comparison
// sort on the block key took ~3 ms per call on the GPU box's host at C4, twice
// per first pass of a context: profiles/r05o/trace_first).
// Entries may carry flag bits outside `key` (the tile-pair list's single
// flag): they ride along, the order is the keyed tiles'.
inline uint32_t super_block_side(uint32_t NP) { return 24ull * 64 * NP <= (4ull << 20) ? 16u : 8u; }
inline std::vector<uint32_t> xcd_order(const std::vector<uint32_t> &t, uint32_t kS, uint32_t key = ~0u) {
    constexpr uint32_t kX = 8;
    std::vector<uint32_t> sorted(t);
    auto keyed_less = [key](uint32_t x, uint32_t y) { return (x & key) < (y & key); };
    if (!std::is_sorted(sorted.begin(), sorted.end(), keyed_less))
        std::sort(sorted.begin(), sorted.end(), keyed_less);
    uint32_t nbr = 0, nbc = 0;
    for (uint32_t v : sorted) {
        v &= key;
        nbr = std::max(nbr, (v >> 16) / kS + 1);
        nbc = std::max(nbc, (v & 0xFFFFu) / kS + 1);
    }
    auto block_of = [&](uint32_t v) {
        v &= key;
        return (size_t)((v >> 16) / kS) * nbc + (v & 0xFFFFu) / kS;
    };
    std::vector<uint32_t> start((size_t)nbr * nbc + 1, 0);
    for (uint32_t v : sorted) ++start[block_of(v) + 1];
    for (size_t b = 1; b < start.size(); ++b) start[b] += start[b - 1];
    std::vector<uint32_t> by_block(sorted.size());
    {
        std::vector<uint32_t> at(start.begin(), start.end() - 1);
        for (uint32_t v : sorted) by_block[at[block_of(v)]++] = v;  // stable: ascending inside a block
    }
    std::vector<std::vector<uint32_t>> q(kX);
    for (size_t b = 0; b + 1 < start.size(); ++b) {
        if (start[b] == start[b + 1]) continue;
        size_t x = 0;
        for (size_t k = 1; k < kX; ++k)
            if (q[k].size() < q[x].size()) x = k;
        q[x].insert(q[x].end(), by_block.begin() + start[b], by_block.begin() + start[b + 1]);
    }
    // Even out the queues to within one tile: the kernel runs in rounds of
    // (resident workgroups per XCD) and a queue a few tiles longer than the
    // others costs a whole extra round (rank 0's 1/8 shard of C4: 7 rounds
    // instead of 6).  Tail tiles move from the longest queue to the shortest.
    for (;;) {
        size_t lo = 0, hi = 0;
        for (size_t k = 1; k < kX; ++k) {
            if (q[k].size() < q[lo].size()) lo = k;
            if (q[k].size() > q[hi].size()) hi = k;
        }
        if (q[hi].size() <= q[lo].size() + 1) break;
        q[lo].push_back(q[hi].back());
        q[hi].pop_back();
    }
    size_t len = 0;
    for (auto &v : q) len = std::max(len, v.size());
    std::vector<uint32_t> out(len * kX, kNoTileEntry);
    for (size_t x = 0; x < kX; ++x)
        for (size_t i = 0; i < q[x].size(); ++i) out[i * kX + x] = q[x][i];
    return out;
}

// The fp6 screen's pair list of a tile list (sorted by (ta, tb)): tiles (ta,
// tb) and (ta, tb + 1) with tb even form an entry ta << 16 | tb; any other
// tile is an entry of its own (kSingleEntry set).  Within a 256-site chunk
// row the pairs never cross a chunk (four tiles per chunk).  Returned in the
// tile list's order of first tiles.
constexpr uint32_t kSingleEntry = 0x8000u;  // (= pair_mfma.hip kF6Single)
inline std::vector<uint32_t> fp6_pair_list(const std::vector<uint32_t> &sorted_tiles) {
    std::vector<uint32_t> out;
    for (size_t i = 0; i < sorted_tiles.size(); ++i) {
        const uint32_t t = sorted_tiles[i];
        if ((t & 1u) == 0 && i + 1 < sorted_tiles.size() && sorted_tiles[i + 1] == t + 1) {
            out.push_back(t);
            ++i;
        } else {
            out.push_back(t | kSingleEntry);
        }
    }
    return out;
}
}  // namespace tile_order
}  // namespace wld
