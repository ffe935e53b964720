// Reference-order assembly of the passing rows.
//
// The pair kernels write each 64x64 tile's passing rows to a staging slice
// taken with one atomic per tile, and record per (site a, 64-wide b tile)
// segment its row count and staging offset, plus per reference chunk
// (256x256, lib.rs:615) its total.  These two kernels turn that into the
// reference's PairStore order (lib.rs:623-683): chunks in triu_index order
// (rows descending, columns ascending), inside a chunk a ascending, then b.
//   chunk_scan: exclusive scan of the shard's chunk totals in linear order
//   gather:     one workgroup per chunk; scans its 256 rows x 4 segments and
//               copies the rows, mapping filtered site indices to parent
//               indices through site_map (lib.rs:662-663).
#include <algorithm>

#include "pair_common.hpp"

namespace wld {

// Zeroes a run's counters, its chunk totals and the segment counts (one launch
// instead of three memsets).
__global__ __launch_bounds__(256) void run_init_kernel(unsigned long long *__restrict__ counters,
                                                        uint32_t *__restrict__ chunk_total, uint32_t n_chunks) {
    const uint32_t i0 = blockIdx.x * 256 + threadIdx.x, stride = gridDim.x * 256;
    if (i0 < kCounterWords) counters[i0] = 0;
    for (uint32_t i = i0; i < n_chunks; i += stride) chunk_total[i] = 0;
}

// host_out (mapped pinned host memory) receives {staging cursor, row total,
// candidate tiles}: the run's only device-to-host transfer, without a copy
// command.  The scan also leaves the run state clean for the next run (the
// staging cursor and the range's chunk totals back to 0), so a run needs no
// initialising kernel.  After a screen it runs in the screen's or the
// candidate launch's last workgroup instead (scan_tail).
__global__ __launch_bounds__(1024) void chunk_scan_kernel(ScanArgs a) { chunk_scan_block(a); }

// inverse of chunk_linear: exact integer version of triu_index (lib.rs:623-632)
__device__ inline void chunk_of_linear(uint32_t n, uint32_t i, uint32_t &row, uint32_t &col) {
    uint32_t rf = (uint32_t)((sqrt(8.0 * (double)i + 1.0) - 1.0) * 0.5);
    while ((uint64_t)(rf + 1) * (rf + 2) / 2 <= i) ++rf;
    while ((uint64_t)rf * (rf + 1) / 2 > i) --rf;
    row = n - rf - 1;
    col = row + i - rf * (rf + 1) / 2;
}

// One workgroup per (chunk, 16-row slice): every slice re-derives the chunk's
// row prefix from the segment counts (256 rows x 4 bytes, one dword per row:
// T is a multiple of 4), then copies only its 16 rows, so a chunk full of rows
// spreads over 16 workgroups.  A chunk without rows (its base equals the
// next chunk's) and a slice without rows leave at once.  The copy issues all
// 16 rows' loads before any store (wave s: b tile s of the chunk, lane e: the
// e-th row of that segment), so a workgroup waits for one round of staging
// loads, not sixteen.
constexpr uint32_t kGatherRows = 16;

__global__ __launch_bounds__(256) void gather_kernel(OrderArgs o, const uint32_t *__restrict__ chunk_base,
                                                      uint32_t lin_begin, uint32_t count, uint32_t n_chunk_rows,
                                                      uint32_t L, uint64_t rows,
                                                      const unsigned long long *__restrict__ state,
                                                      uint64_t out_cap,
                                                      const uint32_t *__restrict__ site_map,
                                                      uint32_t *__restrict__ out_a, uint32_t *__restrict__ out_b,
                                                      float *__restrict__ out_d, float *__restrict__ out_dp,
                                                      float *__restrict__ out_r2) {
    __shared__ uint8_t sCnt[kGatherRows][kTilesPerChunk];
    __shared__ uint32_t sOff[kGatherRows][kTilesPerChunk];
    __shared__ uint32_t sPre[kGatherRows][kTilesPerChunk];
    __shared__ uint32_t sWave[4];
    if (state) {  // enqueued behind the scan, before the host has seen it
        if (state[kCursorSeen] > o.st_capacity || state[1] > out_cap) return;  // (uniform) the host redoes it
        rows = state[1];
    }
    // work items (chunk, 16-row slice), chunk-major, over a capped grid (a
    // grid of every item held the screen of the next step out of its CU
    // slots while both ran): workgroup w's items w, w + G, ...  Which of them
    // lie in chunks with rows is read for up to 256 at once (one round trip,
    // not one per item: linkage-block C4 has rows in a few percent of its
    // 3,160 chunks), and only those are visited (round 6: its order phase
    // 0.054 -> 0.045 ms, the step 1.132 -> 1.125 ms, profiles/r06ac/)
    constexpr uint32_t kSlices = kChunk / kGatherRows;
    __shared__ uint32_t sItems[256], sNum;
    const uint32_t n_items = count * kSlices;
    const uint32_t my_n = n_items > blockIdx.x ? (n_items - blockIdx.x + gridDim.x - 1) / gridDim.x : 0u;
    for (uint32_t kb = 0; kb < my_n; kb += 256) {
    {
        const uint32_t k = kb + threadIdx.x;
        bool any = false;
        if (k < my_n) {
            const uint32_t ci = (blockIdx.x + k * gridDim.x) / kSlices;
            const uint64_t nx = ci + 1 < count ? chunk_base[ci + 1] : rows;
            any = nx != chunk_base[ci];
        }
        if (threadIdx.x == 0) sNum = 0;
        __syncthreads();
        if (any) sItems[atomicAdd(&sNum, 1u)] = k;  // (any order: each item writes its own rows)
        __syncthreads();
    }
    const uint32_t num = sNum;
    for (uint32_t q = 0; q < num; ++q) {
    const uint32_t item = blockIdx.x + sItems[q] * gridDim.x;
    const uint32_t ci = item / kSlices, slice = item % kSlices;
    const uint32_t base = chunk_base[ci];
    const uint32_t lin = lin_begin + ci;
    uint32_t row, col;
    chunk_of_linear(n_chunk_rows, lin, row, col);
    const uint32_t tid = threadIdx.x;
    const uint32_t r0 = slice * kGatherRows;
    const uint32_t a = row * kChunk + tid;
    // the tiles the pair kernel computed (b tile >= a tile, inside L) each
    // wrote their 64 counts; the other bytes of the dword are stale
    uint32_t word = 0;
    if (a < L) word = *reinterpret_cast<const uint32_t *>(o.seg_cnt + (size_t)a * o.T + col * kTilesPerChunk);
    uint32_t cnt[kTilesPerChunk], rowtot = 0;
#pragma unroll
    for (int s = 0; s < kTilesPerChunk; ++s) {
        const uint32_t tb = col * kTilesPerChunk + s;
        cnt[s] = (a < L && tb * kTile < L && tb >= a / kTile) ? (word >> (8 * s)) & 0xFFu : 0u;
        rowtot += cnt[s];
    }
    const uint32_t incl = wave_inclusive_scan(rowtot);
    if ((tid & 63) == 63) sWave[tid >> 6] = incl;
    const uint32_t slice_end = r0 + kGatherRows;
    // the slice's own rows: any?
    if (!__syncthreads_or(tid >= r0 && tid < slice_end && rowtot != 0)) continue;  // (after a barrier: sWave is free)
    if (tid >= r0 && tid < slice_end) {  // this slice's rows
        uint32_t wbase = 0;
        for (uint32_t k = 0; k < (tid >> 6); ++k) wbase += sWave[k];
        uint32_t pre = base + wbase + incl - rowtot;
#pragma unroll
        for (int s = 0; s < kTilesPerChunk; ++s) {
            const uint32_t tb = col * kTilesPerChunk + s;
            sCnt[tid - r0][s] = (uint8_t)cnt[s];
            sOff[tid - r0][s] = cnt[s] ? o.seg_off[(size_t)a * o.T + tb] : 0u;
            sPre[tid - r0][s] = pre;
            pre += cnt[s];
        }
    }
    __syncthreads();
    const uint32_t s = tid >> 6, e = tid & 63;
    uint32_t fa[kGatherRows], fb[kGatherRows];
    float fd[kGatherRows], fdp[kGatherRows], fr2[kGatherRows];
    uint64_t dst[kGatherRows];
    bool has[kGatherRows];
#pragma unroll
    for (uint32_t r = 0; r < kGatherRows; ++r) {
        has[r] = e < sCnt[r][s];
        const uint64_t src = (uint64_t)sOff[r][s] + e;
        dst[r] = (uint64_t)sPre[r][s] + e;
        if (has[r] && (dst[r] >= rows || src >= o.st_capacity)) {  // (the run's counts disagree: not written)
            report_guard(o, kGuardGather);
            has[r] = false;
        }
        if (has[r]) {
            fa[r] = o.st_a[src];
            fb[r] = o.st_b[src];
            fd[r] = o.st_d[src];
            fdp[r] = o.st_dp[src];
            fr2[r] = o.st_r2[src];
        }
    }
#pragma unroll
    for (uint32_t r = 0; r < kGatherRows; ++r) {
        if (!has[r]) continue;
        out_a[dst[r]] = site_map ? site_map[fa[r]] : fa[r];
        out_b[dst[r]] = site_map ? site_map[fb[r]] : fb[r];
        out_d[dst[r]] = fd[r];
        out_dp[dst[r]] = fdp[r];
        out_r2[dst[r]] = fr2[r];
    }
    __syncthreads();  // the slice tables are rewritten by the next item
    }
    __syncthreads();  // (sItems and sNum are rewritten by the next batch)
    }
}

// tiles of each chunk of [lin_begin, lin_begin + count) in the pair kernels'
// lists (b tile >= a tile, inside the set's T_used tiles)
__global__ __launch_bounds__(256) void progress_init_kernel(unsigned *__restrict__ chunk_left, uint32_t lin_begin,
                                                             uint32_t count, uint32_t n_chunk_rows, uint32_t T_used,
                                                             unsigned *__restrict__ prog_n) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i == 0) *prog_n = 0;
    if (i >= count) return;
    uint32_t row, col;
    chunk_of_linear(n_chunk_rows, lin_begin + i, row, col);
    const uint32_t ra = min(T_used - min(T_used, row * kTilesPerChunk), (uint32_t)kTilesPerChunk);
    const uint32_t rb = min(T_used - min(T_used, col * kTilesPerChunk), (uint32_t)kTilesPerChunk);
    chunk_left[lin_begin + i] = (row == col ? ra * (ra + 1) / 2 : ra * rb) * kTileQuarters;  // (tile_done)
}

void launch_progress_init(unsigned *chunk_left, uint32_t lin_begin, uint32_t count, uint32_t n_chunk_rows, uint32_t L,
                          unsigned *prog_n, hipStream_t s) {
    const uint32_t T_used = (L + kTile - 1) / kTile;
    hipLaunchKernelGGL(progress_init_kernel, dim3((std::max<uint32_t>(count, 1) + 255) / 256), dim3(256), 0, s,
                       chunk_left, lin_begin, count, n_chunk_rows, T_used, prog_n);
}

void launch_run_init(unsigned long long *counters, uint32_t *chunk_total, uint32_t n_chunks, hipStream_t s) {
    const unsigned blocks = (unsigned)std::min<size_t>((std::max<size_t>(n_chunks, 4) + 255) / 256, 2048);
    hipLaunchKernelGGL(run_init_kernel, dim3(blocks), dim3(256), 0, s, counters, chunk_total, n_chunks);
}

void launch_chunk_scan(const ScanArgs &a, hipStream_t s) {
    hipLaunchKernelGGL(chunk_scan_kernel, dim3(1), dim3(1024), 0, s, a);
}

void launch_gather(const OrderArgs &o, const uint32_t *chunk_base, uint32_t lin_begin, uint32_t count,
                   uint32_t n_chunk_rows, uint32_t L, uint64_t rows, const unsigned long long *state,
                   uint64_t out_cap, const uint32_t *site_map, uint32_t *out_a, uint32_t *out_b, float *out_d,
                   float *out_dp, float *out_r2, hipStream_t s) {
    if (!count) return;
    // two workgroups per CU at most (C4 at 16 slices per chunk would be 50,560)
    constexpr uint32_t kGatherGrid = 512;
    const uint32_t items = count * (kChunk / kGatherRows);
    hipLaunchKernelGGL(gather_kernel, dim3(std::min(items, kGatherGrid)), dim3(256), 0, s, o, chunk_base, lin_begin,
                       count, n_chunk_rows, L, rows, state, out_cap, site_map, out_a, out_b, out_d, out_dp, out_r2);
}

}  // namespace wld
