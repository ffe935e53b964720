// f32 pair kernel: the exact-f32 path (and the fallback for weights the
// integer MFMA kernel's fixed-point planes cannot hold exactly).  For finite
// weights the products and sums run on f32-input MFMA (MF below); the VALU
// loop described next is the SAFE (non-finite weights) path and the
// WLD_VALU_PLAIN=1 variant.
//
// Replaces the inner loop of single_weighted_ld_pair (lib.rs:416-480) for a
// 64x64 tile of site pairs per 256-thread workgroup.  Each thread owns a 4x4
// block of pairs (a = a0 + ty + 16i, b = b0 + tx + 16j) and keeps the four
// weighted masked sums of lib.rs:441-444 per pair in registers:
//     T   += w  where a in {maj,min} and b in {maj,min}
//     SA  += w  where additionally a == maj
//     SB  += w  where additionally b == maj
//     SAB += w  where a == maj and b == maj
// as fmaf(u, f, acc) with u = w or 0 (a side) and f = 1.0 or 0.0 (b side):
// w*1 and w*0 are exact, so each sum is an f32 sum over sequences in order
// (64-sequence stage sums added into a running total; the same terms in the
// same order for all four sums, so SA == T still implies SAB == SB exactly and
// degenerate pairs stay NaN as in the reference).  (The SAFE variant uses selects, for non-finite weights
// where 0*inf would differ from the reference's select.)  Codes of both 64-site
// panels and the weights are staged through LDS 64 sequences at a time.
#include "pair_common.hpp"

namespace wld {

namespace {
constexpr int kStride = 68;  // LDS row stride in bytes (17 dwords: conflict-free b reads)
}

typedef float v4f __attribute__((ext_vector_type(4)));

// MF = true: the products and f32 sums of the non-SAFE path on the matrix
// cores, v_mfma_f32_16x16x4_f32 (f32 inputs, exact products, an f32 fma chain
// over k: the same terms in the same sequence order as the VALU loop).  Wave w
// owns a rows 16w..16w+15 against the tile's 64 b columns in four 16x16
// blocks; lane l = 16g + r carries a row r (A) / b column r (B) at sequence
// kk + g, and holds the sums of pairs (a = 16w + 4g + e, b = 16n + r) — the
// same thread -> (4 a rows, 4 b columns) shape as the VALU mapping (a = ty +
// 16i), so the epilogue and compaction only change how a row slot maps to a.
// The VALU's code extraction then overlaps the matrix pipe instead of
// competing with the FMAs for VALU issue.
#ifndef WLD_VALU_MF_WG
#define WLD_VALU_MF_WG 2  // MF: 164 VGPRs would fit 3 per CU; measured equal
#endif
template <bool DENSE, bool SAFE, bool MF>
__global__ __launch_bounds__(256, MF ? WLD_VALU_MF_WG : 2) void pair_valu_kernel(const uint8_t *__restrict__ codes,
                                                         const float *__restrict__ w,
                                                         const uint8_t *__restrict__ site_ok,
                                                         const uint32_t *__restrict__ tiles, uint32_t L, uint32_t NP,
                                                         uint32_t flush, uint32_t n_chunk_rows, float thr, OrderArgs o,
                                                         DenseArgs dn) {
    __shared__ __attribute__((aligned(16))) uint8_t sA[kTile * kStride];
    __shared__ __attribute__((aligned(16))) uint8_t sB[kTile * kStride];
    __shared__ __attribute__((aligned(16))) float sW[64];

    const uint32_t tile = tiles[blockIdx.x];
    if (tile == kNoTile) return;  // padding of an XCD-ordered list (whole workgroup)
    const uint32_t ta = tile >> 16, tb = tile & 0xFFFFu;
    const uint32_t a0 = ta * kTile, b0 = tb * kTile;
    const uint32_t tid = threadIdx.x;
    const uint32_t tx = tid & 15, ty = tid >> 4;

    // Two-level summation: acc holds a block of `flush` 64-sequence stages,
    // tot the running total (tot += acc after every block).  A plain running
    // sum over thousands of sequences loses ~N*2^-24 relative (e.g. 5008
    // Henikoff weights of ~0.002 into a total of ~10); the reference's 8 lane
    // sums (lib.rs:418-445) lose N/8*2^-24; blocks of ~sqrt(N) sequences
    // (flush = round(sqrt(NP)/64), launch_pair_valu) leave ~2 sqrt(N)*2^-24.
    float acc[4][4][4], tot[4][4][4];
    v4f accM[4][4];  // MF: [b block n][sum q], element e = a row slot
    // a row of the tile for row slot i of this thread (b = tx + 16 j either way)
    auto arow = [&](int i) -> uint32_t { return MF ? 4 * ty + i : ty + 16 * i; };
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) tot[i][j][q] = 0.0f;

    const uint32_t lr = tid >> 2, part = tid & 3;  // loader: site row, 16-byte part
    const uint8_t *gA = codes + (size_t)(a0 + lr) * NP + part * 16;
    const uint8_t *gB = codes + (size_t)(b0 + lr) * NP + part * 16;

    uint32_t left = 0;  // stages until the next flush of acc into tot
    for (uint32_t k0 = 0; k0 < NP; k0 += 64) {
        const uint4 va = *reinterpret_cast<const uint4 *>(gA + k0);
        const uint4 vb = *reinterpret_cast<const uint4 *>(gB + k0);
        const float wv = tid < 64 ? w[k0 + tid] : 0.0f;
        __syncthreads();
        uint32_t *pa = reinterpret_cast<uint32_t *>(sA + lr * kStride + part * 16);
        uint32_t *pb = reinterpret_cast<uint32_t *>(sB + lr * kStride + part * 16);
        pa[0] = va.x; pa[1] = va.y; pa[2] = va.z; pa[3] = va.w;
        pb[0] = vb.x; pb[1] = vb.y; pb[2] = vb.z; pb[3] = vb.w;
        if (tid < 64) sW[tid] = wv;
        __syncthreads();
        if (left == 0) {
            left = flush;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        acc[i][j][q] = 0.0f;
                        accM[j][q][i] = 0.0f;
                    }
        }

        if constexpr (MF) {
            const uint32_t lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
            const uint8_t *rowA = sA + (16 * wave + r) * kStride + g;
            const uint8_t *rowB = sB + r * kStride + g;
#pragma unroll 4
            for (int kk = 0; kk < 64; kk += 4) {
                const float we = sW[kk + g];
                const uint32_t ca = rowA[kk];
                const float u = (ca & kCodeIn) ? we : 0.0f;
                const float v = (ca & kCodeMaj) ? we : 0.0f;
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    const uint32_t cb = rowB[16 * n * kStride + kk];
                    const float fi = (float)(cb & 1u), fm = (float)(cb >> 1);
                    accM[n][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(u, fi, accM[n][0], 0, 0, 0);
                    accM[n][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(v, fi, accM[n][1], 0, 0, 0);
                    accM[n][2] = __builtin_amdgcn_mfma_f32_16x16x4f32(u, fm, accM[n][2], 0, 0, 0);
                    accM[n][3] = __builtin_amdgcn_mfma_f32_16x16x4f32(v, fm, accM[n][3], 0, 0, 0);
                }
            }
        } else

#pragma unroll 2
        for (int kk = 0; kk < 64; kk += 4) {
            uint32_t A[4], B[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) A[i] = *reinterpret_cast<const uint32_t *>(sA + (ty + 16 * i) * kStride + kk);
#pragma unroll
            for (int j = 0; j < 4; ++j) B[j] = *reinterpret_cast<const uint32_t *>(sB + (tx + 16 * j) * kStride + kk);
            const float4 w4 = *reinterpret_cast<const float4 *>(sW + kk);
            const float wk[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float we = wk[e];
                float u[4], v[4];
                uint32_t ca[4], cb[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    ca[i] = (A[i] >> (8 * e)) & 3u;
                    u[i] = (ca[i] & kCodeIn) ? we : 0.0f;
                    v[i] = (ca[i] & kCodeMaj) ? we : 0.0f;
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) cb[j] = (B[j] >> (8 * e)) & 3u;
                if constexpr (!SAFE) {
                    float fi[4], fm[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        fi[j] = (float)(cb[j] & 1u);
                        fm[j] = (float)(cb[j] >> 1);
                    }
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            acc[i][j][0] = __builtin_fmaf(u[i], fi[j], acc[i][j][0]);
                            acc[i][j][1] = __builtin_fmaf(v[i], fi[j], acc[i][j][1]);
                            acc[i][j][2] = __builtin_fmaf(u[i], fm[j], acc[i][j][2]);
                            acc[i][j][3] = __builtin_fmaf(v[i], fm[j], acc[i][j][3]);
                        }
                } else {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const bool bi = cb[j] & 1u, bm = cb[j] & 2u;
                            acc[i][j][0] += bi ? u[i] : 0.0f;
                            acc[i][j][1] += bi ? v[i] : 0.0f;
                            acc[i][j][2] += bm ? u[i] : 0.0f;
                            acc[i][j][3] += bm ? v[i] : 0.0f;
                        }
                }
            }
        }
        if (--left == 0 || k0 + 64 >= NP) {
            left = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int q = 0; q < 4; ++q) tot[i][j][q] += MF ? accM[j][q][i] : acc[i][j][q];
        }
    }

    // ---- epilogue ------------------------------------------------------
    uint32_t passmask[4] = {0, 0, 0, 0};  // bit j per row i
    float res[4][4][3];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t a = a0 + arow(i);
        const bool oka = a < L && site_ok[a];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t b = b0 + tx + 16 * j;
            float d, dp, r2;
            ld_epilogue(tot[i][j][0], tot[i][j][1], tot[i][j][2], tot[i][j][3], d, dp, r2);
            res[i][j][0] = d;
            res[i][j][1] = dp;
            res[i][j][2] = r2;
            const bool valid = oka && a < b && b < L && site_ok[b];
            if constexpr (DENSE) {
                if (a < b && b < L) {
                    const size_t k = (size_t)a * L + b;
                    dn.d[k] = d;
                    dn.dp[k] = dp;
                    dn.r2[k] = r2;
                    dn.valid[k] = valid ? 1 : 0;
                }
            } else {
                if (valid && r2 > thr) passmask[i] |= 1u << j;  // lib.rs:660 strict '>'
            }
        }
    }
    if constexpr (DENSE) return;

    // ---- compaction: rows of each a in b order, tile slice of the staging ----
    __shared__ uint8_t sMask[kTile][16];
    __shared__ uint16_t sRowM[kTile][4];
    __shared__ uint16_t sRowP[kTile][4];
    __shared__ uint32_t sRowBase[kTile];
#pragma unroll
    for (int i = 0; i < 4; ++i) sMask[arow(i)][tx] = (uint8_t)passmask[i];
    __syncthreads();
    if (tid < kTile) {
        const uint32_t r = tid;
        uint32_t M[4] = {0, 0, 0, 0};
        for (int x = 0; x < 16; ++x) {
            const uint32_t nib = sMask[r][x];
#pragma unroll
            for (int j = 0; j < 4; ++j) M[j] |= ((nib >> j) & 1u) << x;
        }
        uint32_t p = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            sRowM[r][j] = (uint16_t)M[j];
            sRowP[r][j] = (uint16_t)p;
            p += __popc(M[j]);
        }
        const uint32_t cnt = p;
        const uint32_t incl = wave_inclusive_scan(cnt);
        const uint32_t excl = incl - cnt;
        const uint32_t total = __shfl(incl, 63, 64);
        unsigned long long base = 0;
        if (r == 63 && total) base = atomicAdd(o.cursor, (unsigned long long)total);
        base = __shfl(base, 63, 64);
        sRowBase[r] = (uint32_t)base + excl;
        const uint32_t a = a0 + r;
        o.seg_cnt[(size_t)a * o.T + tb] = (uint8_t)cnt;
        o.seg_off[(size_t)a * o.T + tb] = (uint32_t)base + excl;
        if (r == 63 && total)
            atomicAdd(&o.chunk_total[chunk_linear(n_chunk_rows, ta / kTilesPerChunk, tb / kTilesPerChunk)], total);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (!passmask[i]) continue;
        const uint32_t r = arow(i);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (!(passmask[i] & (1u << j))) continue;
            const uint64_t pos = (uint64_t)sRowBase[r] + sRowP[r][j] + __popc(sRowM[r][j] & ((1u << tx) - 1u));
            if (pos < o.st_capacity) {
                o.st_a[pos] = a0 + r;
                o.st_b[pos] = b0 + tx + 16 * j;
                o.st_d[pos] = res[i][j][0];
                o.st_dp[pos] = res[i][j][1];
                o.st_r2[pos] = res[i][j][2];
            }
        }
    }
}

void launch_pair_valu(const uint8_t *codes, const float *w, const uint8_t *site_ok, const uint32_t *tiles,
                      uint32_t n_tiles, uint32_t L, uint32_t NP, uint32_t n_chunk_rows, float thr, bool safe,
                      bool plain, const OrderArgs &o, const DenseArgs *dense, hipStream_t s) {
    DenseArgs dn = dense ? *dense : DenseArgs{nullptr, nullptr, nullptr, nullptr};
    const uint32_t flush = (uint32_t)std::max(1.0, std::floor(std::sqrt((double)NP) / 64.0 + 0.5));
    // finite weights: products and sums on the matrix cores (plain, option
    // WLD_OPT_VALU_PLAIN: the VALU loop, for A/B); non-finite weights keep the
    // select loop
    const dim3 g(n_tiles), b(256);
    if (dense) {
        if (safe)
            hipLaunchKernelGGL((pair_valu_kernel<true, true, false>), g, b, 0, s, codes, w, site_ok, tiles, L, NP,
                               flush, n_chunk_rows, thr, o, dn);
        else if (plain)
            hipLaunchKernelGGL((pair_valu_kernel<true, false, false>), g, b, 0, s, codes, w, site_ok, tiles, L, NP,
                               flush, n_chunk_rows, thr, o, dn);
        else
            hipLaunchKernelGGL((pair_valu_kernel<true, false, true>), g, b, 0, s, codes, w, site_ok, tiles, L, NP,
                               flush, n_chunk_rows, thr, o, dn);
    } else {
        if (safe)
            hipLaunchKernelGGL((pair_valu_kernel<false, true, false>), g, b, 0, s, codes, w, site_ok, tiles, L, NP,
                               flush, n_chunk_rows, thr, o, dn);
        else if (plain)
            hipLaunchKernelGGL((pair_valu_kernel<false, false, false>), g, b, 0, s, codes, w, site_ok, tiles, L, NP,
                               flush, n_chunk_rows, thr, o, dn);
        else
            hipLaunchKernelGGL((pair_valu_kernel<false, false, true>), g, b, 0, s, codes, w, site_ok, tiles, L, NP,
                               flush, n_chunk_rows, thr, o, dn);
    }
}

}  // namespace wld
