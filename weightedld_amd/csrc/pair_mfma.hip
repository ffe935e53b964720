// Exact-integer MFMA pair kernel (the default path).
//
// The four masked weighted sums of single_weighted_ld_pair (lib.rs:416-480)
//     T   = sum_k w_k in_a[k]  in_b[k]      SA  = sum_k w_k maj_a[k] in_b[k]
//     SB  = sum_k w_k in_a[k]  maj_b[k]     SAB = sum_k w_k maj_a[k] maj_b[k]
// are, over all site pairs at once, the product X_A diag(w) X_B^T of 0/1
// "in"/"major" indicator matrices (in = symbol is the site's major or minor,
// lib.rs:435; maj = symbol is the major, lib.rs:430-432) — a dense contraction
// over the sequence axis.  It runs on the int8 matrix cores:
//   * weights become fixed point q_k = rint(w_k * 2^shift), |q_k| < 2^23, split
//     into three balanced base-256 digits d_p in [-128,127]
//     (q = d0 + 256 d1 + 65536 d2; built once per load by mfma_prep_kernel);
//   * A operand (a sites): indicator byte & digit byte  (in & d_p, maj & d_p);
//     B operand (b sites): indicator bytes 0/1;
//   * 12 v_mfma_i32_32x32x32_i8 per 32 sequences accumulate the 2x3x2
//     (channel_a, plane, channel_b) partial sums in int32, exactly;
//   * epilogue: S = sum_p 2^(8p) acc_p in int64 (exact), converted once to f32
//     (correctly rounded: the f32 the reference's sum would be without its
//     rounding error), then the reference epilogue (lib.rs:482-520) in f32.
// Exact integer sums keep the reference's degenerate-pair behaviour exactly:
// SA == T implies SAB == SB, so monomorphic-in-mask pairs give 0/0 = NaN and
// are dropped by the strict r2 > threshold (lib.rs:660).
//
// Tiling: a 256-thread workgroup owns a 64x64 tile of site pairs (the tile
// list is the triangular set of (a-tile, b-tile) with b-tile >= a-tile of the
// shard's chunk rows); each wave owns a 32x32 sub-tile and streams its 32 a-
// and 32 b-site code rows (16 bytes per lane per 32 sequences) straight from
// HBM/L2 into registers.  Passing rows are compacted per 64x64 tile in LDS
// exactly like the VALU kernel (order.hip assembles the reference order).
#include "pair_common.hpp"

namespace wld {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

bool mfma_supported() { return true; }

// digit planes [3][NP] int8 of q = rint(w * 2^shift)
__global__ __launch_bounds__(256) void mfma_prep_kernel(const float *__restrict__ w_pad, uint32_t NP, int shift,
                                                         int8_t *__restrict__ planes) {
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= NP) return;
    long long q = llrint(ldexp((double)w_pad[k], shift));
    int d[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        long long r = ((q + 128) & 255) - 128;  // balanced digit in [-128, 127]
        d[p] = (int)r;
        q = (q - r) / 256;
    }
    planes[k] = (int8_t)d[0];
    planes[NP + k] = (int8_t)d[1];
    planes[2 * NP + k] = (int8_t)d[2];
}

__device__ __forceinline__ v16i mfma_i8(v4i a, v4i b, v16i c) {
    return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
}

template <bool DENSE>
__global__ __launch_bounds__(256, 2) void pair_mfma_kernel(const uint8_t *__restrict__ codes,
                                                            const int8_t *__restrict__ planes,
                                                            const uint8_t *__restrict__ site_ok,
                                                            const uint32_t *__restrict__ tiles, uint32_t L,
                                                            uint32_t NP, uint32_t n_chunk_rows, float thr, int shift,
                                                            OrderArgs o, DenseArgs dn) {
    const uint32_t tile = tiles[blockIdx.x];
    const uint32_t ta = tile >> 16, tb = tile & 0xFFFFu;
    const uint32_t a0 = ta * kTile, b0 = tb * kTile;
    const uint32_t tid = threadIdx.x;
    const uint32_t wave = tid >> 6, lane = tid & 63;
    const uint32_t wa = wave >> 1, wb = wave & 1;
    const uint32_t r = lane & 31, h = lane >> 5;

    const uint8_t *pa = codes + (size_t)(a0 + 32 * wa + r) * NP + 16 * h;
    const uint8_t *pb = codes + (size_t)(b0 + 32 * wb + r) * NP + 16 * h;
    const int8_t *pd = planes + 16 * h;

    v16i acc[2][3][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int y = 0; y < 2; ++y)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[x][p][y][e] = 0;

    v4i ca = *reinterpret_cast<const v4i *>(pa);
    v4i cb = *reinterpret_cast<const v4i *>(pb);
    v4i d0 = *reinterpret_cast<const v4i *>(pd);
    v4i d1 = *reinterpret_cast<const v4i *>(pd + NP);
    v4i d2 = *reinterpret_cast<const v4i *>(pd + 2 * NP);
    for (uint32_t k0 = 0; k0 < NP; k0 += 32) {
        // prefetch the next 32 sequences while this block's MFMAs run
        const uint32_t kn = (k0 + 32 < NP) ? k0 + 32 : k0;
        const v4i na = *reinterpret_cast<const v4i *>(pa + kn);
        const v4i nb = *reinterpret_cast<const v4i *>(pb + kn);
        const v4i n0 = *reinterpret_cast<const v4i *>(pd + kn);
        const v4i n1 = *reinterpret_cast<const v4i *>(pd + NP + kn);
        const v4i n2 = *reinterpret_cast<const v4i *>(pd + 2 * NP + kn);

        const v4i one = {0x01010101, 0x01010101, 0x01010101, 0x01010101};
        const v4i b_in = cb & one;
        const v4i b_maj = (cb >> 1) & one;
        const v4i a_in = (ca & one) * 0xFF;         // 0x00 / 0xFF byte masks
        const v4i a_maj = ((ca >> 1) & one) * 0xFF;
        const v4i dp[3] = {d0, d1, d2};
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            const v4i ai = a_in & dp[p];
            const v4i am = a_maj & dp[p];
            acc[0][p][0] = mfma_i8(ai, b_in, acc[0][p][0]);
            acc[0][p][1] = mfma_i8(ai, b_maj, acc[0][p][1]);
            acc[1][p][0] = mfma_i8(am, b_in, acc[1][p][0]);
            acc[1][p][1] = mfma_i8(am, b_maj, acc[1][p][1]);
        }
        ca = na;
        cb = nb;
        d0 = n0;
        d1 = n1;
        d2 = n2;
    }

    // ---- epilogue: lane holds b = b0+32wb+r and 16 a rows -------------------
    const double scale = ldexp(1.0, -shift);
    const uint32_t b_local = 32 * wb + r;
    const uint32_t b = b0 + b_local;
    const bool okb = b < L && site_ok[b];
    float res[16][3];
    uint32_t pass = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t a_local = 32 * wa + (i & 3) + 8 * (i >> 2) + 4 * h;
        const uint32_t a = a0 + a_local;
        float s[2][2];
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y) {
                const long long v = (long long)acc[x][0][y][i] + ((long long)acc[x][1][y][i] << 8) +
                                    ((long long)acc[x][2][y][i] << 16);
                s[x][y] = (float)((double)v * scale);
            }
        float d, dp, r2;
        ld_epilogue(s[0][0], s[1][0], s[0][1], s[1][1], d, dp, r2);
        res[i][0] = d;
        res[i][1] = dp;
        res[i][2] = r2;
        const bool valid = okb && a < b && site_ok[a];
        if constexpr (DENSE) {
            if (a < b && b < L) {
                const size_t k = (size_t)a * L + b;
                dn.d[k] = d;
                dn.dp[k] = dp;
                dn.r2[k] = r2;
                dn.valid[k] = valid ? 1 : 0;
            }
        } else {
            if (valid && r2 > thr) pass |= 1u << i;  // lib.rs:660 strict '>'
        }
    }
    if constexpr (DENSE) return;

    // ---- compaction: a 64x64 pass-bit matrix in LDS, rows in b order ----------
    __shared__ unsigned long long sBits[kTile];
    __shared__ uint32_t sRowBase[kTile];
    if (tid < kTile) sBits[tid] = 0ull;
    __syncthreads();
    if (pass) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (pass & (1u << i)) {
                const uint32_t a_local = 32 * wa + (i & 3) + 8 * (i >> 2) + 4 * h;
                atomicOr(&sBits[a_local], 1ull << b_local);
            }
    }
    __syncthreads();
    if (tid < kTile) {
        const uint32_t rr = tid;
        const uint32_t cnt = __popcll(sBits[rr]);
        const uint32_t incl = wave_inclusive_scan(cnt);
        const uint32_t excl = incl - cnt;
        const uint32_t total = __shfl(incl, 63, 64);
        unsigned long long base = 0;
        if (rr == 63 && total) base = atomicAdd(o.cursor, (unsigned long long)total);
        base = __shfl(base, 63, 64);
        sRowBase[rr] = (uint32_t)base + excl;
        const uint32_t a = a0 + rr;
        o.seg_cnt[(size_t)a * o.T + tb] = (uint8_t)cnt;
        o.seg_off[(size_t)a * o.T + tb] = (uint32_t)base + excl;
        if (rr == 63 && total)
            atomicAdd(&o.chunk_total[chunk_linear(n_chunk_rows, ta / kTilesPerChunk, tb / kTilesPerChunk)], total);
    }
    __syncthreads();
    if (pass) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if (!(pass & (1u << i))) continue;
            const uint32_t a_local = 32 * wa + (i & 3) + 8 * (i >> 2) + 4 * h;
            const uint64_t pos =
                (uint64_t)sRowBase[a_local] + __popcll(sBits[a_local] & ((1ull << b_local) - 1ull));
            if (pos < o.st_capacity) {
                o.st_a[pos] = a0 + a_local;
                o.st_b[pos] = b;
                o.st_d[pos] = res[i][0];
                o.st_dp[pos] = res[i][1];
                o.st_r2[pos] = res[i][2];
            }
        }
    }
}

void launch_mfma_prep(const uint8_t *, const float *w_pad, size_t, size_t NP, int shift, int8_t *planes,
                      hipStream_t s) {
    hipLaunchKernelGGL(mfma_prep_kernel, dim3((unsigned)((NP + 255) / 256)), dim3(256), 0, s, w_pad, (uint32_t)NP,
                       shift, planes);
}

void launch_pair_mfma(const uint8_t *codes, const int8_t *wplanes, const uint8_t *site_ok, const uint32_t *tiles,
                      uint32_t n_tiles, uint32_t L, uint32_t NP, uint32_t n_chunk_rows, float thr, int shift,
                      const OrderArgs &o, const DenseArgs *dense, hipStream_t s) {
    if (dense)
        hipLaunchKernelGGL((pair_mfma_kernel<true>), dim3(n_tiles), dim3(256), 0, s, codes, wplanes, site_ok, tiles, L,
                           NP, n_chunk_rows, thr, shift, o, *dense);
    else
        hipLaunchKernelGGL((pair_mfma_kernel<false>), dim3(n_tiles), dim3(256), 0, s, codes, wplanes, site_ok, tiles,
                           L, NP, n_chunk_rows, thr, shift, o, DenseArgs{nullptr, nullptr, nullptr, nullptr});
}

}  // namespace wld
