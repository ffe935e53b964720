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
//   * A operand (a sites): the digit where the indicator is set (in & d_p,
//     maj & d_p); B operand (b sites): indicator bytes 0/1;
//   * 48 v_mfma_i32_16x16x64_i8 per 64 sequences and wave accumulate the
//     2x3x2 (channel_a, plane, channel_b) partial sums of 16x64 site pairs in
//     int32, exactly (the 16x16 shape holds a higher clock under load than
//     32x32x32 at the same cycles per op: C5 -9%, C4 -5% measured);
//   * epilogue: S = sum_p 2^(8p) acc_p, exact in f64, converted once to f32
//     (correctly rounded: the f32 the reference's sum would be without its
//     rounding error), then the reference epilogue (lib.rs:482-520) in f32.
// Exact integer sums keep the reference's degenerate-pair behaviour exactly:
// SA == T implies SAB == SB, so monomorphic-in-mask pairs give 0/0 = NaN and
// are dropped by the strict r2 > threshold (lib.rs:660).
//
// Work decomposition: the pair space is cut into 64x64 site tiles (the
// triangular list of (a-tile, b-tile), b-tile >= a-tile, of the shard's chunk
// rows); a 256-thread workgroup computes a tile, wave w its a rows 16w..16w+15
// against all 64 b columns (each digit-masked A operand feeds 8 MFMAs: 56
// v_perm per 48 MFMAs, against 64 for 32x32 wave tiles); two workgroups share
// a CU, so one's epilogue and first-group latency overlap the other's matrix
// work.  Operands stream through LDS in groups of kGroup 32-sequence stages
// (read back two stages = 64 sequences at a time), double-buffered and filled
// by LDS-DMA
// (global_load_lds_dwordx4, async, no VGPRs): per stage each wave copies one
// 1 KB code-fragment block (A0, A1, B0, B1 of the fragment-major layout) and
// per group wave 0 the group's 1 KB of weight digits.  Every DMA is a
// full-wave 1 KB copy, and a group is consumed only after s_waitcnt vmcnt(0)
// by every issuing wave + a barrier — correctness never depends on the
// completion order of outstanding loads; a buffer is refilled only after the
// barrier that follows its readers' s_waitcnt lgkmcnt(0).  The next group is
// issued right after the barrier and lands during this group's 4 x 48 MFMAs.
// Passing rows are compacted per tile in LDS (order.hip assembles the
// reference order).
#include "pair_common.hpp"


namespace wld {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

bool mfma_supported() { return true; }

namespace {
constexpr int kGroup = 8;                           // 32-sequence stages per LDS group
constexpr int kStageCodes = 4096;                   // A0 A1 B0 B1, 1 KB each
constexpr int kDigStage = 128;                      // digit bytes per stage: [plane][half][16] + 32 pad
constexpr int kDigGroup = 1024;                     // digit records of one group: one full-wave DMA
// stages per LDS group of the kernel with NPL active digit planes: one plane
// (equal weights) uses 4-stage groups, 34 KB of LDS per workgroup and 108
// VGPRs, so four workgroups (4 waves per SIMD) share a CU
#ifndef WLD_KG1
#define WLD_KG1 4
#endif
#ifndef WLD_WG1
#define WLD_WG1 (WLD_KG1 <= 4 ? 4 : 2)
#endif
template <int NPL>
struct GroupShape {
    static constexpr int kStages = NPL == 1 ? WLD_KG1 : kGroup;
    static constexpr int kBytes = kStages * kStageCodes + kDigGroup;
    static constexpr int kWgPerCu = NPL == 1 ? WLD_WG1 : 2;
};

__host__ __device__ inline size_t digf_offset(size_t NP) { return 3 * NP; }
__host__ __device__ inline size_t okbits_offset(size_t NP) {
    return 3 * NP + (NP / 32 + kGroup - 1) / kGroup * kDigGroup;
}
// byte of the digit record of stage kb within digf
__host__ __device__ inline size_t digf_stage(uint32_t kb) { return (size_t)(kb / kGroup) * kDigGroup + (kb % kGroup) * kDigStage; }
}  // namespace

// planes buffer (mfma_planes_bytes): the weight digits of q = rint(w * 2^shift)
// in two layouts, then the site filter as bits:
//   planes[p*NP + k]                      plane-major (site-major kernel path)
//   digf[(kb/kGroup)*1024 + (kb%kGroup)*128 + (2p + h)*16 + j]
//                                         per 32-sequence stage, 1 KB per group
//                                         (LDS path; k = 32kb + 16h + j)
//   ok_bits[g] bit i = site 64g+i passes  (site_ok, lib.rs:400-408)
//   plane_mask (u32 after the bits)       bit p = some digit of plane p is nonzero
__host__ __device__ inline size_t planemask_offset(size_t LP, size_t NP) { return okbits_offset(NP) + LP / 64 * 8; }
// + 1 KB: a half-group (kg < kGroup) digit DMA copies 1 KB from a 512-B offset
size_t mfma_planes_bytes(size_t LP, size_t NP) { return planemask_offset(LP, NP) + 16 + kDigGroup; }

__global__ __launch_bounds__(256) void mfma_prep_kernel(const float *__restrict__ w_pad, uint32_t NP, int shift,
                                                         int8_t *__restrict__ planes, int8_t *__restrict__ digf,
                                                         unsigned *__restrict__ plane_mask) {
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= NP) return;
    unsigned used = 0;
    long long q = llrint(ldexp((double)w_pad[k], shift));
    const uint32_t kb = k >> 5, h = (k >> 4) & 1, j = k & 15;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        const long long r = ((q + 128) & 255) - 128;  // balanced digit in [-128, 127]
        q = (q - r) / 256;
        planes[p * NP + k] = (int8_t)r;
        digf[digf_stage(kb) + (2 * p + h) * 16 + j] = (int8_t)r;
        used |= (r != 0) << p;
    }
    if (used) atomicOr(plane_mask, used);
}

// one wave per 64 sites
__global__ __launch_bounds__(64) void okbits_kernel(const uint8_t *__restrict__ site_ok, uint32_t L,
                                                     uint64_t *__restrict__ ok_bits) {
    const uint32_t s = blockIdx.x * 64 + threadIdx.x;
    const uint64_t m = __ballot(s < L && site_ok[s]);
    if (threadIdx.x == 0) ok_bits[blockIdx.x] = m;
}

// codes_frag: the (site, sequence) codes in "fragment-major" order, so a
// wave's A or B operand for 32 sites x 32 sequences is one contiguous 1 KB
// block (lane l = 32h + r gets site r, sequences 16h..16h+15 — the MFMA
// operand layout):
//   frag[((g * NKB + kb) * 64 + l) * 16 + j] = sel(codes[(32g + (l&31)) * NP + 32kb + 16(l>>5) + j])
// Each byte is stored as a v_perm_b32 selector for its byte position j&3:
//   12 (not major/minor -> constant 0x00), j&3 (minor), 4 + (j&3) (major),
// so one v_perm_b32 per dword turns codes + weight digits straight into MFMA
// operands (mfma_block_sel) with no mask arithmetic.
__global__ __launch_bounds__(256) void frag_kernel(const uint8_t *__restrict__ codes, uint32_t LP, uint32_t NP,
                                                    uint8_t *__restrict__ frag) {
    const uint32_t NKB = NP / 32;
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;  // one 16-byte chunk
    if (idx >= (size_t)LP * NP / 16) return;
    const uint32_t l = idx & 63;
    const size_t t = idx >> 6;
    const uint32_t kb = t % NKB;
    const size_t g = t / NKB;
    const uint4 v = *reinterpret_cast<const uint4 *>(codes + (g * 32 + (l & 31)) * NP + kb * 32 + (l >> 5) * 16);
    uint32_t in[4] = {v.x, v.y, v.z, v.w}, out[4], raw[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        uint32_t o = 0, r = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t c = (in[e] >> (8 * j)) & 0xFF;
            const uint32_t sel = (c & kCodeIn) ? ((c & kCodeMaj) ? 4u + j : (uint32_t)j) : 12u;
            o |= sel << (8 * j);
            r |= ((c & kCodeIn) ? ((c & kCodeMaj) ? 2u : 1u) : 0u) << (8 * j);
        }
        out[e] = o;
        raw[e] = r;
    }
    *reinterpret_cast<uint4 *>(frag + idx * 16) = make_uint4(out[0], out[1], out[2], out[3]);
    // the B-side copy: 0 (not major/minor), 1 (minor), 2 (major) = minor + 2 major
    *reinterpret_cast<uint4 *>(frag + (size_t)LP * NP + idx * 16) = make_uint4(raw[0], raw[1], raw[2], raw[3]);
}

__device__ __forceinline__ v16i mfma_i8(v4i a, v4i b, v16i c) {
    return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ v4i mfma_i8_16(v4i a, v4i b, v4i c) {
    return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
}

// A wave's share of the 64x64 tile as (channel_a, plane, channel_b) int32
// sums, and where its 16 (a, b) pairs per lane sit (MFMA C/D layouts, gfx950).
// 32x32x32 shape, wave w owns the 32x32 sub-tile (w >> 1, w & 1): lane
// (r, h) = (lane & 31, lane >> 5) holds b = r and a = (i & 3) + 8 (i >> 2) + 4h.
template <int NPL>
struct Acc32 {
    static constexpr int kPlanes = NPL;
    v16i v[2][NPL][2];  // [channel_a][plane][channel_b]
    __device__ __forceinline__ int get(int x, int p, int y, int i) const { return v[x][p][y][i]; }
    static __device__ __forceinline__ uint32_t a_local(int i, uint32_t wave, uint32_t lane) {
        return 32 * (wave >> 1) + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
    }
    static __device__ __forceinline__ uint32_t b_local(int i, uint32_t wave, uint32_t lane) {
        return 32 * (wave & 1) + (lane & 31);
    }
};
// 16x16x64 shape, wave w owns a rows 16w..16w+15 against all 64 b columns as
// four 16x16 blocks n (C/D col = lane & 15, row = 4 (lane >> 4) + e); register
// i = 4n + e.  NPL = the weight-digit planes that are not all zero (3 for
// general weights, 1 for equal weights, e.g. --unweighted).
template <int NPL>
struct Acc16 {
    static constexpr int kPlanes = NPL;
    v4i v[4][2][NPL][2];  // [n][channel_a][plane][channel_b]
#ifdef WLD_BPERM
    __device__ __forceinline__ int get(int x, int p, int y, int i) const { return v[i >> 2][x][p][y][i & 3]; }
#else
    // channel_b slots hold X = S(raw) = S(minor) + 2 S(major) and Y = S(minor)
    // (mfma_block_sel16): S(in) = (X + Y) / 2, S(major) = (X - Y) / 2, both
    // exact (X - Y is even) and in int32 range (|X| + |Y| <= 3 * 128 NP)
    __device__ __forceinline__ int get(int x, int p, int y, int i) const {
        const int X = v[i >> 2][x][p][0][i & 3], Y = v[i >> 2][x][p][1][i & 3];
        return (y ? X - Y : X + Y) >> 1;
    }
#endif
    static __device__ __forceinline__ uint32_t a_local(int i, uint32_t wave, uint32_t lane) {
        return 16 * wave + 4 * (lane >> 4) + (i & 3);
    }
    static __device__ __forceinline__ uint32_t b_local(int i, uint32_t wave, uint32_t lane) {
        return 16 * (i >> 2) + (lane & 15);
    }
};

// The same 12 products for 64 sequences with v_mfma_i32_16x16x64_i8: the
// wave's 16 a sites (ca) against the tile's 64 b sites in four 16-column
// blocks (cb[n]).  Lane group g = lane >> 4 carries sequences 16g..16g+15 in
// A, B and the digits alike, so the products pair the same sequence whatever
// the k order inside the instruction.  48 MFMAs of 16 cycles = the 24 of 32 of
// two 32x32 stages; each A operand (digit x channel) feeds 8 MFMAs, so it
// takes 56 v_perm per 48 MFMAs (64 with a 32x32 wave tile).
template <int NPL>
__device__ __forceinline__ void mfma_block_sel16(v4i (&acc)[4][2][NPL][2], v4i ca, const v4i (&cb)[4],
                                                 const v4i (&dp)[NPL]) {
    constexpr unsigned kOnes = 0x01010101u;
    v4i b_in[4], b_maj[4];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
#ifdef WLD_BPERM  // selector-coded B: in / major indicators, two v_perm per dword
            b_in[n][e] = (int)__builtin_amdgcn_perm(kOnes, kOnes, (unsigned)cb[n][e]);
            b_maj[n][e] = (int)__builtin_amdgcn_perm(kOnes, 0u, (unsigned)cb[n][e]);
#else  // 0/1/2-coded B: the raw bytes (minor + 2 major) and the minor bit, one v_and per dword
            b_in[n][e] = cb[n][e];
            b_maj[n][e] = cb[n][e] & (int)kOnes;
#endif
        }
#pragma unroll
    for (int p = 0; p < NPL; ++p) {
        v4i ai, am;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            ai[e] = (int)__builtin_amdgcn_perm((unsigned)dp[p][e], (unsigned)dp[p][e], (unsigned)ca[e]);
            am[e] = (int)__builtin_amdgcn_perm((unsigned)dp[p][e], 0u, (unsigned)ca[e]);
        }
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            acc[n][0][p][0] = mfma_i8_16(ai, b_in[n], acc[n][0][p][0]);
            acc[n][0][p][1] = mfma_i8_16(ai, b_maj[n], acc[n][0][p][1]);
            acc[n][1][p][0] = mfma_i8_16(am, b_in[n], acc[n][1][p][0]);
            acc[n][1][p][1] = mfma_i8_16(am, b_maj[n], acc[n][1][p][1]);
        }
    }
}

// Byte-wise masks from raw code bytes c in {0 (out), 1 (minor), 3 (major)}
// (site-major path): v_perm_b32 with zero sources returns, per selector byte,
// 0xFF for >= 13 and 0x00 for 8..12 — a byte compare without a multiply.
__device__ __forceinline__ v4i mask_in(v4i c) {  // c+12 in {12,13,15}: 00 FF FF
    v4i m;
#pragma unroll
    for (int e = 0; e < 4; ++e) m[e] = (int)__builtin_amdgcn_perm(0u, 0u, (unsigned)c[e] | 0x0C0C0C0Cu);
    return m;
}
__device__ __forceinline__ v4i mask_maj(v4i c) {  // c+10 in {10,11,13}: 00 00 FF
    v4i m;
#pragma unroll
    for (int e = 0; e < 4; ++e) m[e] = (int)__builtin_amdgcn_perm(0u, 0u, (unsigned)c[e] + 0x0A0A0A0Au);
    return m;
}

// 12 MFMAs of one 32-sequence block from raw site-major codes
__device__ __forceinline__ void mfma_block(v16i (&acc)[2][3][2], v4i ca, v4i cb, v4i d0, v4i d1, v4i d2) {
    const v4i one = {0x01010101, 0x01010101, 0x01010101, 0x01010101};
    const v4i b_in = cb & one;
    const v4i b_maj = (cb >> 1) & one;
    const v4i a_in = mask_in(ca);
    const v4i a_maj = mask_maj(ca);
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
}

// One full-wave LDS-DMA (global_load_lds_dwordx4): each lane copies 16 bytes
// from gsrc to LDS byte address lds_dst + 16*lane (lds_dst wave-uniform).  Issued
// as inline asm so that the compiler's wait-count bookkeeping does not see it
// (it would otherwise wait for every in-flight copy before any LDS read of the
// other buffer): completion is ordered only by the kernel's own protocol —
// s_waitcnt vmcnt(0) by every issuing wave, then a barrier, then the reads.
// M0 is saved and restored inside the statement (it is compiler-reserved).
__device__ __forceinline__ void glds16(const void *gsrc, uint32_t lds_dst) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds_dst)
        : "memory");
}

__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

#ifdef WLD_EXP_STAMPS
// diagnostic build only: per-tile cycle stamps of wave 0 (start, first group,
// loop end, epilogue end) and where it ran (HW_ID | XCC_ID << 32)
constexpr unsigned kStampWords = 5;
__device__ unsigned long long g_stamps[kStampWords << 18];
__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
extern "C" int wld_debug_stamps_copy(unsigned long long *out, unsigned n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), (size_t)n * kStampWords * 8) == hipSuccess ? 0 : -1;
}
#endif

template <int NPL>
__device__ __forceinline__ void zero_acc(Acc32<NPL> &acc) {
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int p = 0; p < NPL; ++p)
#pragma unroll
            for (int y = 0; y < 2; ++y)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc.v[x][p][y][e] = 0;
}
template <int NPL>
__device__ __forceinline__ void zero_acc(Acc16<NPL> &acc) {
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int p = 0; p < NPL; ++p)
#pragma unroll
                for (int y = 0; y < 2; ++y)
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc.v[n][x][p][y][e] = 0;
}

// Reference epilogue of one pair from its exact sums (fixed-point units):
// the optional exact-algebra prefilter, then lib.rs:482-520 in f32.  Returns
// true when the pair passes (valid and r2 > thr, lib.rs:660); d/dp/r2 are
// written when the f32 epilogue ran (always for DENSE).
template <bool DENSE, bool PREFILTER>
__device__ __forceinline__ bool pair_eval(double T, double SA, double SB, double SAB, bool valid, float thr,
                                          double scale, float &d, float &dp, float &r2) {
    if constexpr (!DENSE) {
        if (!valid) return false;
        if constexpr (PREFILTER) {
            // Exact algebra: d = PA*PB - P(AB) and r2 = d^2/(PA Pa PB Pb) become
            // r2 = (SA*SB - SAB*T)^2 / (SA (T-SA) SB (T-SB)) on the exact sums.
            // Evaluated in f64 (|err| ~1e-16 relative); pairs more than
            // 1e-5 + 1e-4|thr| below the threshold cannot pass the f32 epilogue,
            // so they skip it.  Everything else (and den <= 0, the NaN/inf
            // cases) takes the full reference epilogue.
            const double num = SA * SB - SAB * T;
            const double den = SA * (T - SA) * SB * (T - SB);
            const double cut = (double)thr - (1e-5 + 1e-4 * fabs((double)thr));
            if (den > 0.0 && num * num < cut * den) return false;
        }
    }
    ld_epilogue((float)(T * scale), (float)(SA * scale), (float)(SB * scale), (float)(SAB * scale), d, dp, r2);
    return valid && r2 > thr;
}

// Epilogue of one 64x64 tile.  The lane holds b = b0 + 32wb + r and 16 a rows
// (MFMA C layout: row (i&3) + 8(i>>2) + 4h).  DENSE writes every pair's stats
// (tests); otherwise passing pairs are compacted through the tile's 64x64
// pass-bit matrix in LDS into staging, with per-(a, b-tile) segment counts and
// offsets for order.hip.  PREFILTER (threshold > 0) skips the f32 epilogue for
// pairs whose exact r2, evaluated in f64 from the exact sums, lies clearly
// below the threshold.
template <bool DENSE, bool PREFILTER, class Acc>
__device__ __forceinline__ void tile_epilogue(const Acc &acc, uint32_t ta, uint32_t tb, uint32_t tid,
                                              uint64_t okA, uint64_t okB, uint32_t L, uint32_t n_chunk_rows,
                                              float thr, int shift, bool narrow, uint32_t plane_idx,
                                              const OrderArgs &o, const DenseArgs &dn, unsigned long long *sBits,
                                              uint32_t *sRowBase) {
    const uint32_t wave = tid >> 6, lane = tid & 63;
    double pscale[Acc::kPlanes];  // 2^(8 idx_j) of the j-th active plane (plane_idx: 2 bits per plane)
#pragma unroll
    for (int j = 0; j < Acc::kPlanes; ++j) pscale[j] = (double)(1u << (8 * ((plane_idx >> (2 * j)) & 3)));
    const uint32_t a0 = ta * kTile, b0 = tb * kTile;
    const double scale = ldexp(1.0, -shift);
    float res[16][3];
    uint32_t pass = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t a_local = Acc::a_local(i, wave, lane);
        const uint32_t b_local = Acc::b_local(i, wave, lane);
        const uint32_t a = a0 + a_local, b = b0 + b_local;
        const bool valid = ((okB >> b_local) & 1) && a < b && ((okA >> a_local) & 1);
#ifdef WLD_EXP_NOEPI
        if constexpr (!DENSE) {  // diagnostic: accumulators consumed, no epilogue arithmetic
            int x = 0;
#pragma unroll
            for (int c = 0; c < 4 * Acc::kPlanes; ++c)
                x ^= acc.get(c / (2 * Acc::kPlanes), (c / 2) % Acc::kPlanes, c % 2, i);
            if (valid && x == 0x7fffffff) pass |= 1u << i;
            res[i][0] = res[i][1] = res[i][2] = 0.f;
            continue;
        }
#endif
        // S = acc_0 + 2^8 acc_1 + 2^16 acc_2: integers below 2^48, exact in f64.
        // |acc_p| <= 128 NP, so acc_1 + 2^8 acc_2 is exact in int32 while
        // 32896 NP < 2^31 (NP <= 65024): one int op, two conversions, one FMA.
        // With fewer planes (all-zero digit planes skipped) S = sum_j 2^(8 idx_j) acc_j.
        double S[2][2];
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y) {
                if constexpr (Acc::kPlanes < 3) {
                    double v = 0.0;
#pragma unroll
                    for (int j = 0; j < Acc::kPlanes; ++j) v = fma(pscale[j], (double)acc.get(x, j, y, i), v);
                    S[x][y] = v;
                } else if (narrow) {
                    const int hi = acc.get(x, 1, y, i) + acc.get(x, 2, y, i) * 256;
                    S[x][y] = fma(256.0, (double)hi, (double)acc.get(x, 0, y, i));
                } else {
                    S[x][y] = fma(65536.0, (double)acc.get(x, 2, y, i),
                                  fma(256.0, (double)acc.get(x, 1, y, i), (double)acc.get(x, 0, y, i)));
                }
            }
        float d = 0.f, dp = 0.f, r2 = 0.f;
        const bool ok = pair_eval<DENSE, PREFILTER>(S[0][0], S[1][0], S[0][1], S[1][1], valid, thr, scale, d, dp, r2);
        res[i][0] = d;
        res[i][1] = dp;
        res[i][2] = r2;
        if constexpr (DENSE) {
            if (a < b && b < L) {
                const size_t k = (size_t)a * L + b;
                dn.d[k] = d;
                dn.dp[k] = dp;
                dn.r2[k] = r2;
                dn.valid[k] = valid ? 1 : 0;
            }
        } else {
            if (ok) pass |= 1u << i;  // lib.rs:660 strict '>'
        }
    }
    if constexpr (DENSE) return;

    // ---- compaction: a 64x64 pass-bit matrix in LDS, rows in b order ----------
    // A tile with no passing pair (every tile at the bench threshold on random
    // data) writes only its 64 zero counts (seg_off is read only where
    // seg_cnt > 0).  One barrier decides it.
    if (!__syncthreads_or(pass != 0)) {
        if (tid < kTile) o.seg_cnt[(size_t)(a0 + tid) * o.T + tb] = 0;
        return;
    }
    if (tid < kTile) sBits[tid] = 0ull;
    __syncthreads();
    if (pass) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (pass & (1u << i))
                atomicOr(&sBits[Acc::a_local(i, wave, lane)], 1ull << Acc::b_local(i, wave, lane));
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
            const uint32_t a_local = Acc::a_local(i, wave, lane);
            const uint32_t b_local = Acc::b_local(i, wave, lane);
            const uint64_t pos =
                (uint64_t)sRowBase[a_local] + __popcll(sBits[a_local] & ((1ull << b_local) - 1ull));
            if (pos < o.st_capacity) {
                o.st_a[pos] = a0 + a_local;
                o.st_b[pos] = b0 + b_local;
                o.st_d[pos] = res[i][0];
                o.st_dp[pos] = res[i][1];
                o.st_r2[pos] = res[i][2];
            }
        }
    }
}

// LDS-streaming kernel over fragment-major, selector-coded codes: one 64x64
// tile per workgroup.  (An XCD-contiguous block->tile remap measured no gain:
// the 41 MB code copy of BASELINE config 4 is served from L2/MALL either way.)
template <bool DENSE, bool PREFILTER, int NPL>
__global__ __launch_bounds__(256, GroupShape<NPL>::kWgPerCu) void pair_mfma_kernel(const uint8_t *__restrict__ frag,
                                                            const uint8_t *__restrict__ frag_b,
                                                            const int8_t *__restrict__ planes,
                                                            const uint64_t *__restrict__ ok_bits,
                                                            const uint32_t *__restrict__ tiles, uint32_t L,
                                                            uint32_t NP, uint32_t n_chunk_rows, float thr, int shift,
                                                            uint32_t plane_idx, OrderArgs o, DenseArgs dn) {
    constexpr int KG = GroupShape<NPL>::kStages, KGB = GroupShape<NPL>::kBytes;
    __shared__ __attribute__((aligned(16))) uint8_t smem[2 * KGB];  // operand groups (DMA targets)
    __shared__ unsigned long long sBits[kTile];                              // compaction (never a DMA target)
    __shared__ uint32_t sRowBase[kTile];

    const uint32_t tid = threadIdx.x;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const uint32_t NKB = NP / 32;
    const uint32_t n_groups = (NKB + KG - 1) / KG;

#ifdef WLD_EXP_STAMPS
    const unsigned long long ts0 = stamp();
#endif
    const uint32_t tile = tiles[blockIdx.x];
    if (tile == kNoTile) return;  // padding of an XCD-ordered list (whole workgroup)
    const uint32_t ta = tile >> 16, tb = tile & 0xFFFFu;

    // this wave's 1 KB code block per stage: A0/A1 (a sites), B0/B1 (b sites)
    const uint32_t g = wave < 2 ? 2 * ta + wave : 2 * tb + (wave - 2);
#ifdef WLD_BPERM
    (void)frag_b;
    const uint8_t *src = frag + (size_t)g * NKB * 1024;  // wave-uniform
#else
    const uint8_t *src = (wave < 2 ? frag : frag_b) + (size_t)g * NKB * 1024;  // wave-uniform
#endif
    const int8_t *digf = planes + digf_offset(NP);
    const uint32_t smem_lds = lds_addr(smem);
    auto issue = [&](uint32_t grp, uint32_t buf) {
        const uint32_t gb = smem_lds + buf * KGB;
        const uint32_t kb0 = grp * KG;
        const uint8_t *base = src + (size_t)kb0 * 1024;
        const uint32_t lane16 = lane * 16;
#pragma unroll
        for (int st = 0; st < KG; ++st)
            if (kb0 + st < NKB) glds16(base + (uint32_t)(st * 1024) + lane16, gb + st * kStageCodes + wave * 1024);
        // digit records of the group's stages (128 B each, contiguous from
        // digf_stage(kb0)): one 1 KB full-wave copy (allocation padded past
        // the last group)
        if (wave == 0) glds16(digf + digf_stage(kb0) + lane16, gb + KG * kStageCodes);
    };

    issue(0, 0);
    const uint64_t okA = ok_bits[ta], okB = ok_bits[tb];
    Acc16<NPL> acc;
    // lane group g = lane >> 4 reads stage 2s + (g >> 1), half g & 1, of each
    // 64-sequence step (the 32-stage fragment layout, re-addressed): a sites
    // 16w.. = rows 16(w & 1).. of 32-site block w >> 1; b block n = rows
    // 16(n & 1).. of B block n >> 1
    const uint32_t g4 = lane >> 4, so = g4 >> 1, hh = g4 & 1;
    const uint32_t lrow = so * kStageCodes + (32 * hh + (lane & 15)) * 16;
    const uint32_t offA = lrow + (wave >> 1) * 1024 + (wave & 1) * 256;
    const uint32_t offB = lrow + 2048;  // + (n >> 1) * 1024 + (n & 1) * 256
    const uint32_t offD = KG * kStageCodes + so * kDigStage + hh * 16;
    // the active planes' 32-byte rows of a stage's digit record (all three:
    // compile-time offsets, so the reads keep immediate offsets)
    uint32_t offP[NPL];
#pragma unroll
    for (int j = 0; j < NPL; ++j) offP[j] = NPL == 3 ? offD + 32 * j : offD + 32 * ((plane_idx >> (2 * j)) & 3);
    zero_acc(acc);
    uint32_t buf = 0;
#ifdef WLD_EXP_PRIO
    __builtin_amdgcn_s_setprio(WLD_EXP_PRIO);  // the matrix loop outranks a partner's epilogue VALU
#endif
#ifdef WLD_EXP_STAMPS
    unsigned long long tsg = 0;
#endif
    for (uint32_t grp = 0; grp < n_groups; ++grp) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's copies of this group landed
        __builtin_amdgcn_s_barrier();                     // ... and every other wave's; the other buffer is free
        asm volatile("" ::: "memory");
#ifdef WLD_EXP_STAMPS
        if (grp == 0) tsg = stamp();
#endif
        if (grp + 1 < n_groups) issue(grp + 1, buf ^ 1);
        const uint8_t *gb = smem + buf * KGB;
        const uint32_t n_st = min((uint32_t)KG, NKB - grp * KG);
        for (uint32_t st = 0; st < n_st; st += 2) {  // n_st is even: NP is a multiple of 64
            const uint8_t *sc = gb + st * kStageCodes;
            const uint8_t *sd = gb + st * kDigStage;
            const v4i ca = *reinterpret_cast<const v4i *>(sc + offA);
            const v4i cb[4] = {*reinterpret_cast<const v4i *>(sc + offB), *reinterpret_cast<const v4i *>(sc + offB + 256),
                               *reinterpret_cast<const v4i *>(sc + offB + 1024),
                               *reinterpret_cast<const v4i *>(sc + offB + 1280)};
            v4i dp[NPL];
#pragma unroll
            for (int j = 0; j < NPL; ++j)
                dp[j] = *reinterpret_cast<const v4i *>(NPL == 3 ? sd + offD + 32 * j : sd + offP[j]);
            mfma_block_sel16<NPL>(acc.v, ca, cb, dp);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads of this buffer done before the next barrier
        buf ^= 1;
    }
#ifdef WLD_EXP_STAMPS
    const unsigned long long ts1 = stamp();
#endif
#ifdef WLD_EXP_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
    tile_epilogue<DENSE, PREFILTER>(acc, ta, tb, tid, okA, okB, L, n_chunk_rows, thr, shift, NP <= 65024u,
                                    plane_idx, o, dn, sBits, sRowBase);
#ifdef WLD_EXP_STAMPS
    const unsigned long long ts2 = stamp();
    if (tid == 0 && blockIdx.x < (1u << 18)) {
        const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_REG_HW_ID
        const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));  // HW_REG_XCC_ID
        g_stamps[kStampWords * blockIdx.x] = ts0;
        g_stamps[kStampWords * blockIdx.x + 1] = tsg;
        g_stamps[kStampWords * blockIdx.x + 2] = ts1;
        g_stamps[kStampWords * blockIdx.x + 3] = ts2;
        g_stamps[kStampWords * blockIdx.x + 4] = hw | ((unsigned long long)xcc << 32);
    }
#endif
}

// Site-major variant (one tile per workgroup, codes read straight into
// registers): the reference for the LDS path's race screen and the
// WLD_MFMA_LAYOUT=rows experiments.
template <bool DENSE, bool PREFILTER>
__global__ __launch_bounds__(256, 2) void pair_mfma_rows_kernel(const uint8_t *__restrict__ codes,
                                                                 const int8_t *__restrict__ planes,
                                                                 const uint64_t *__restrict__ ok_bits,
                                                                 const uint32_t *__restrict__ tiles, uint32_t L,
                                                                 uint32_t NP, uint32_t n_chunk_rows, float thr,
                                                                 int shift, OrderArgs o, DenseArgs dn) {
    __shared__ unsigned long long sBits[kTile];
    __shared__ uint32_t sRowBase[kTile];
    const uint32_t tile = tiles[blockIdx.x];
    if (tile == kNoTile) return;  // padding of an XCD-ordered list (whole workgroup)
    const uint32_t ta = tile >> 16, tb = tile & 0xFFFFu;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t wa = wave >> 1, wb = wave & 1, r = lane & 31, h = lane >> 5;
    Acc32<3> acc;
    zero_acc(acc);
    const uint8_t *pa = codes + (size_t)(ta * kTile + 32 * wa + r) * NP + 16 * h;
    const uint8_t *pb = codes + (size_t)(tb * kTile + 32 * wb + r) * NP + 16 * h;
    const int8_t *pd = planes + 16 * h;
    for (uint32_t k0 = 0; k0 < NP; k0 += 32) {
        const v4i ca = *reinterpret_cast<const v4i *>(pa + k0);
        const v4i cb = *reinterpret_cast<const v4i *>(pb + k0);
        const v4i d0 = *reinterpret_cast<const v4i *>(pd + k0);
        const v4i d1 = *reinterpret_cast<const v4i *>(pd + NP + k0);
        const v4i d2 = *reinterpret_cast<const v4i *>(pd + 2 * NP + k0);
        mfma_block(acc.v, ca, cb, d0, d1, d2);
    }
    tile_epilogue<DENSE, PREFILTER>(acc, ta, tb, tid, ok_bits[ta], ok_bits[tb], L, n_chunk_rows, thr, shift,
                                    NP <= 65024u, 0x24u, o, dn, sBits, sRowBase);
}

void launch_mfma_prep(const uint8_t *site_ok, const float *w_pad, size_t L, size_t LP, size_t NP, int shift,
                      int8_t *planes, hipStream_t s) {
    unsigned *mask = reinterpret_cast<unsigned *>(planes + planemask_offset(LP, NP));
    (void)hipMemsetAsync(mask, 0, sizeof(unsigned), s);
    hipLaunchKernelGGL(mfma_prep_kernel, dim3((unsigned)((NP + 255) / 256)), dim3(256), 0, s, w_pad, (uint32_t)NP,
                       shift, planes, planes + digf_offset(NP), mask);
    hipLaunchKernelGGL(okbits_kernel, dim3((unsigned)(LP / 64)), dim3(64), 0, s, site_ok, (uint32_t)L,
                       reinterpret_cast<uint64_t *>(planes + okbits_offset(NP)));
}

void launch_frag(const uint8_t *codes, size_t LP, size_t NP, uint8_t *frag, hipStream_t s) {
    const size_t chunks = LP * NP / 16;
    hipLaunchKernelGGL(frag_kernel, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0, s, codes, (uint32_t)LP,
                       (uint32_t)NP, frag);
}

template <int NPL>
void launch_lds(const uint8_t *frag, const uint8_t *frag_b, const int8_t *wplanes, const uint64_t *ok_bits, const uint32_t *tiles,
                uint32_t n_tiles, uint32_t L, uint32_t NP, uint32_t n_chunk_rows, float thr, int shift,
                uint32_t plane_idx, bool prefilter, const OrderArgs &o, const DenseArgs *dense, hipStream_t s) {
    const DenseArgs dn = dense ? *dense : DenseArgs{nullptr, nullptr, nullptr, nullptr};
    const dim3 g(n_tiles), b(256);
    if (dense)
        hipLaunchKernelGGL((pair_mfma_kernel<true, false, NPL>), g, b, 0, s, frag, frag_b, wplanes, ok_bits, tiles, L,
                           NP, n_chunk_rows, thr, shift, plane_idx, o, dn);
    else if (prefilter)
        hipLaunchKernelGGL((pair_mfma_kernel<false, true, NPL>), g, b, 0, s, frag, frag_b, wplanes, ok_bits, tiles, L,
                           NP, n_chunk_rows, thr, shift, plane_idx, o, dn);
    else
        hipLaunchKernelGGL((pair_mfma_kernel<false, false, NPL>), g, b, 0, s, frag, frag_b, wplanes, ok_bits, tiles, L,
                           NP, n_chunk_rows, thr, shift, plane_idx, o, dn);
}

unsigned mfma_plane_mask(const int8_t *wplanes, size_t LP, size_t NP, hipStream_t s) {
    unsigned m = 7;
    if (hipMemcpyAsync(&m, wplanes + planemask_offset(LP, NP), sizeof(m), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return 7;  // all planes: always correct
    return m & 7;
}

void launch_pair_mfma(const uint8_t *codes, const uint8_t *frag, const uint8_t *frag_b, const int8_t *wplanes, const uint32_t *tiles,
                      uint32_t n_tiles, uint32_t L, uint32_t NP, uint32_t n_chunk_rows, float thr, int shift,
                      unsigned plane_mask, bool prefilter, const OrderArgs &o, const DenseArgs *dense,
                      hipStream_t s) {
    const DenseArgs dn = dense ? *dense : DenseArgs{nullptr, nullptr, nullptr, nullptr};
    const uint64_t *ok_bits = reinterpret_cast<const uint64_t *>(wplanes + okbits_offset(NP));
    const dim3 g(n_tiles), b(256);
    if (frag) {
        // the nonzero digit planes in ascending order, 2 bits each; no plane is
        // all zero only if some weight is nonzero, which the caller guarantees
        plane_mask &= 7;
        if (!plane_mask) plane_mask = 7;
        uint32_t idx = 0, n = 0;
        for (uint32_t p = 0; p < 3; ++p)
            if (plane_mask >> p & 1) idx |= p << (2 * n++);
        if (n == 3)
            launch_lds<3>(frag, frag_b, wplanes, ok_bits, tiles, n_tiles, L, NP, n_chunk_rows, thr, shift, idx, prefilter, o,
                          dense, s);
        else if (n == 2)
            launch_lds<2>(frag, frag_b, wplanes, ok_bits, tiles, n_tiles, L, NP, n_chunk_rows, thr, shift, idx, prefilter, o,
                          dense, s);
        else
            launch_lds<1>(frag, frag_b, wplanes, ok_bits, tiles, n_tiles, L, NP, n_chunk_rows, thr, shift, idx, prefilter, o,
                          dense, s);
    } else {
        if (dense)
            hipLaunchKernelGGL((pair_mfma_rows_kernel<true, false>), g, b, 0, s, codes, wplanes, ok_bits, tiles, L,
                               NP, n_chunk_rows, thr, shift, o, dn);
        else if (prefilter)
            hipLaunchKernelGGL((pair_mfma_rows_kernel<false, true>), g, b, 0, s, codes, wplanes, ok_bits, tiles, L,
                               NP, n_chunk_rows, thr, shift, o, dn);
        else
            hipLaunchKernelGGL((pair_mfma_rows_kernel<false, false>), g, b, 0, s, codes, wplanes, ok_bits, tiles, L,
                               NP, n_chunk_rows, thr, shift, o, dn);
    }
}

}  // namespace wld
