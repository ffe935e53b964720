// Host check of the run tile lists (weightedld_amd/csrc/tile_order.hpp, used by
// capi.hip build_tiles) against a direct restatement of the round-4 builder:
// tiles generated chunk by chunk in the linear order then sorted; the XCD
// order by a comparison sort on the super-block key; the tile-pair list's
// single flags stripped for the ordering and restored by lookup.  Same lists,
// element for element, for whole sets and shards of several sizes.
#include <cmath>
#include <cstdio>
#include "tile_order.hpp"

using namespace wld::tile_order;

static void chunk_of_linear(uint32_t n, uint32_t i, uint32_t &row, uint32_t &col) {
    uint32_t rf = (uint32_t)((std::sqrt(8.0 * (double)i + 1.0) - 1.0) * 0.5);
    while ((uint64_t)(rf + 1) * (rf + 2) / 2 <= i) ++rf;
    while ((uint64_t)rf * (rf + 1) / 2 > i) --rf;
    row = n - rf - 1;
    col = row + i - rf * (rf + 1) / 2;
}

static std::vector<uint32_t> ref_tiles(uint32_t n, uint32_t T_used, uint32_t lb, uint32_t le) {
    std::vector<uint32_t> t;
    for (uint32_t i = lb; i < le; ++i) {
        uint32_t row, col;
        chunk_of_linear(n, i, row, col);
        for (uint32_t ta = row * 4; ta < std::min<uint32_t>((row + 1) * 4, T_used); ++ta)
            for (uint32_t tb = std::max(ta, col * 4); tb < std::min<uint32_t>((col + 1) * 4, T_used); ++tb)
                t.push_back((ta << 16) | tb);
    }
    std::sort(t.begin(), t.end());
    return t;
}

static std::vector<uint32_t> ref_xcd(const std::vector<uint32_t> &t, uint32_t kS) {
    constexpr uint32_t kX = 8;
    std::vector<uint32_t> sorted(t);
    auto block_of = [kS](uint32_t v) { return ((v >> 16) / kS) << 16 | ((v & 0xFFFFu) / kS); };
    std::sort(sorted.begin(), sorted.end(), [&](uint32_t x, uint32_t y) {
        const uint32_t bx = block_of(x), by = block_of(y);
        return bx != by ? bx < by : x < y;
    });
    std::vector<std::vector<uint32_t>> blocks;
    uint64_t last = ~0ull;
    for (uint32_t v : sorted) {
        if (block_of(v) != last) blocks.emplace_back(), last = block_of(v);
        blocks.back().push_back(v);
    }
    std::vector<std::vector<uint32_t>> q(kX);
    for (auto &b : blocks) {
        size_t x = 0;
        for (size_t k = 1; k < kX; ++k)
            if (q[k].size() < q[x].size()) x = k;
        q[x].insert(q[x].end(), b.begin(), b.end());
    }
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

static std::vector<uint32_t> pair_list(const std::vector<uint32_t> &t) {  // (pair_mfma.hip fp6_pair_list)
    std::vector<uint32_t> out;
    for (size_t i = 0; i < t.size(); ++i) {
        if ((t[i] & 1u) == 0 && i + 1 < t.size() && t[i + 1] == t[i] + 1) {
            out.push_back(t[i]);
            ++i;
        } else {
            out.push_back(t[i] | 0x8000u);
        }
    }
    return out;
}

int main() {
    struct Case { uint32_t L, shards, shard, kS; } cases[] = {
        {20000, 1, 0, 16}, {20000, 8, 0, 16}, {20000, 8, 7, 16}, {20000, 2, 1, 16}, {20000, 4, 2, 8},
        {50000, 1, 0, 8},  {50000, 8, 5, 8},  {2000, 1, 0, 16},  {777, 1, 0, 16},   {33333, 3, 2, 8},
        {300, 1, 0, 16},   {64, 1, 0, 16},    {65, 1, 0, 16},    {12345, 5, 4, 16}};
    int bad = 0;
    for (const auto &c : cases) {
        const uint32_t n = (c.L + 255) / 256, T_used = (c.L + 63) / 64, tot = n * (n + 1) / 2;
        const uint32_t lb = (uint32_t)((uint64_t)tot * c.shard / c.shards);
        const uint32_t le = (uint32_t)((uint64_t)tot * (c.shard + 1) / c.shards);
        const auto t_ref = ref_tiles(n, T_used, lb, le), t = range_tiles(n, T_used, lb, le);
        bool ok = t == t_ref;
        ok = ok && xcd_order(t, c.kS) == ref_xcd(t_ref, c.kS);
        // the tile-pair list: ordered with its flags in place vs stripped and restored
        const auto pl = pair_list(t);
        std::vector<uint32_t> plain(pl.size()), single;
        for (size_t i = 0; i < pl.size(); ++i) {
            plain[i] = pl[i] & ~0x8000u;
            if (pl[i] & 0x8000u) single.push_back(plain[i]);
        }
        std::sort(single.begin(), single.end());
        auto pl_ref = ref_xcd(plain, c.kS);
        for (auto &v : pl_ref)
            if (v != kNoTileEntry && std::binary_search(single.begin(), single.end(), v)) v |= 0x8000u;
        ok = ok && xcd_order(pl, c.kS, ~0x8000u) == pl_ref;
        printf("L=%u shard %u/%u kS=%u: %zu tiles, %zu pair entries: %s\n", c.L, c.shard, c.shards, c.kS, t.size(),
               pl.size(), ok ? "same" : "DIFFERENT");
        bad += !ok;
    }
    printf(bad ? "FAIL\n" : "OK\n");
    return bad ? 1 : 0;
}
