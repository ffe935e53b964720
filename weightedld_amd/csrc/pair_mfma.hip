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
#include <algorithm>
#include <vector>

#include "pair_common.hpp"


namespace wld {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

bool mfma_supported() { return true; }

namespace {
constexpr int kGroup = 8;                           // 32-sequence stages per LDS group
constexpr int kStageCodes = 4096;                   // A0 A1 B0 B1, 1 KB each
constexpr int kDigStage = 128;                      // digit bytes per stage: [plane][half][16], 4 planes
constexpr int kMaxPlanes = 4;                       // balanced base-256 digits of the fixed-point weights
constexpr uint32_t kPlanes012 = 0 | (1 << 2) | (2 << 4);  // plane_idx of planes 0, 1, 2
constexpr int kDigGroup = 1024;                     // digit records of one group: one full-wave DMA
// Shape of the LDS kernel with NPL active digit planes.  One plane (equal
// weights, and the screen) uses 4-stage groups, 34 KB of LDS per workgroup
// and ~108 VGPRs, so four workgroups (4 waves per SIMD) share a CU.  Two or
// three planes: 8-stage groups, four waves of 16 a rows x 64 b columns (NB = 4
// column blocks each), 192 accumulators, two workgroups per CU.  Four planes
// (31-bit fixed point): eight waves of 16 a rows x 32 b columns (NB = 2), so
// the 4 x 32 products per wave fit the same 128 accumulators as two planes
// and no partial sum has to be held across passes; one workgroup per CU,
// still two waves per SIMD.
template <int NPL>
struct GroupShape {
    static constexpr int kStages = NPL == 1 ? 4 : kGroup;
    static constexpr int kBytes = kStages * kStageCodes + kDigGroup;
    static constexpr int kWaves = NPL == 4 ? 8 : 4;
    static constexpr int kNB = NPL == 4 ? 2 : 4;  // 16-column b blocks per wave
    static constexpr int kWgPerCu = NPL == 1 ? 4 : NPL == 4 ? 1 : 2;
};

__host__ __device__ inline size_t digf_offset(size_t NP) { return kMaxPlanes * NP; }
__host__ __device__ inline size_t okbits_offset(size_t NP) {
    return kMaxPlanes * NP + (NP / 32 + kGroup - 1) / kGroup * kDigGroup;
}
// byte of the digit record of stage kb within digf
__host__ __device__ inline size_t digf_stage(uint32_t kb) { return (size_t)(kb / kGroup) * kDigGroup + (kb % kGroup) * kDigStage; }
}  // namespace

// planes buffer (mfma_planes_bytes): the weight digits of q = rint(w * 2^shift)
// (q = d0 + 2^8 d1 + 2^16 d2 + 2^24 d3, balanced digits in [-128, 127]; d3 = 0
// for a 3-plane shift) in two layouts, then the site filter as bits:
//   planes[p*NP + k]                      plane-major (site-major kernel path)
//   digf[(kb/kGroup)*1024 + (kb%kGroup)*128 + (2p + h)*16 + j]
//                                         per 32-sequence stage, 1 KB per group
//                                         (LDS path; k = 32kb + 16h + j)
//   ok_bits[g] bit i = site 64g+i passes  (site_ok, lib.rs:400-408)
//   stats (after the bits, 64 bytes):
//     u32  bit p (p < 4) = some digit of plane p is nonzero; bit 8 = some weight < 0
//     u64  resid[t-1] = sum_k |q_k - 2^(8t) d_t,k| for t = 1, 2, 3: what the top
//          plane t alone leaves out (the screen's residual bound)
//     u64  dsum[p] = sum_k |d_p,k| for p = 0..3 (bounds the screen's sums)
__host__ __device__ inline size_t planemask_offset(size_t LP, size_t NP) { return okbits_offset(NP) + LP / 64 * 8; }
// + 1 KB: a half-group (kg < kGroup) digit DMA copies 1 KB from a 512-B offset
size_t mfma_planes_bytes(size_t LP, size_t NP) { return planemask_offset(LP, NP) + 64 + kDigGroup; }

__global__ __launch_bounds__(256) void mfma_prep_kernel(const float *__restrict__ w_pad, uint32_t NP, int shift,
                                                         int8_t *__restrict__ planes, int8_t *__restrict__ digf,
                                                         unsigned *__restrict__ stats) {
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    unsigned used = 0, res[3] = {0, 0, 0}, ds[kMaxPlanes] = {0, 0, 0, 0};
    if (k < NP) {
        const float w = w_pad[k];
        long long q = llrint(ldexp((double)w, shift));
        const uint32_t kb = k >> 5, h = (k >> 4) & 1, j = k & 15;
        int low = 0;  // q mod 2^(8p), balanced: what planes >= p leave out
#pragma unroll
        for (int p = 0; p < kMaxPlanes; ++p) {
            if (p > 0) res[p - 1] = (unsigned)abs(low);
            const long long r = ((q + 128) & 255) - 128;  // balanced digit in [-128, 127]
            q = (q - r) / 256;
            low += (int)r << (8 * p);
            planes[p * NP + k] = (int8_t)r;
            ds[p] = (unsigned)(r < 0 ? -r : r);
            digf[digf_stage(kb) + (2 * p + h) * 16 + j] = (int8_t)r;
            used |= (r != 0) << p;
        }
        used |= (w < 0.0f) << 8;
    }
    // per-wave sums (<= 64 * 2^23 < 2^32), one atomic each per wave
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        used |= __shfl_xor(used, off, 64);
#pragma unroll
        for (int t = 0; t < 3; ++t) res[t] += __shfl_xor(res[t], off, 64);
#pragma unroll
        for (int p = 0; p < kMaxPlanes; ++p) ds[p] += __shfl_xor(ds[p], off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        if (used) atomicOr(stats, used);
        unsigned long long *acc = reinterpret_cast<unsigned long long *>(stats + 2);
#pragma unroll
        for (int t = 0; t < 3; ++t)
            if (res[t]) atomicAdd(acc + t, (unsigned long long)res[t]);
#pragma unroll
        for (int p = 0; p < kMaxPlanes; ++p)
            if (ds[p]) atomicAdd(acc + 3 + p, (unsigned long long)ds[p]);
    }
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
    static constexpr int kPairs = 16;
    v16i v[2][NPL][2];  // [channel_a][plane][channel_b]
    __device__ __forceinline__ int get(int x, int p, int y, int i) const { return v[x][p][y][i]; }
    static __device__ __forceinline__ uint32_t a_local(int i, uint32_t wave, uint32_t lane) {
        return 32 * (wave >> 1) + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
    }
    static __device__ __forceinline__ uint32_t b_local(int i, uint32_t wave, uint32_t lane) {
        return 32 * (wave & 1) + (lane & 31);
    }
};
// 16x16 sub-block (a_local / 16, b_local / 16) of pair i as a bit index 0..15
template <class Acc>
__device__ __forceinline__ uint32_t sub_block(int i, uint32_t wave, uint32_t lane) {
    return 4 * (Acc::a_local(i, wave, lane) >> 4) + (Acc::b_local(i, wave, lane) >> 4);
}
// 16x16x64 shape, wave w owns a rows 16(w & 3)..+15 against NB 16x16 blocks
// of b columns starting at block NB (w >> 2) (all 64 columns when NB = 4 with
// four waves; 32 when NB = 2 with eight) (C/D col = lane & 15, row =
// 4 (lane >> 4) + e); register i = 4n + e, kPairs = 4 NB per lane.  NPL = the
// weight-digit planes that are not all zero (3 for general weights, 1 for
// equal weights, e.g. --unweighted, 4 for weights spanning more than 2^4).
template <int NPL, int NB = 4>
struct Acc16 {
    static constexpr int kPlanes = NPL;
    static constexpr int kPairs = 4 * NB;
    v4i v[NB][2][NPL][2];  // [n][channel_a][plane][channel_b]
    // channel_b slots hold X = S(raw) = S(minor) + 2 S(major) and Y = S(minor)
    // (mfma_block_sel16): S(in) = (X + Y) / 2, S(major) = (X - Y) / 2, both
    // exact (X - Y is even) and in int32 range (|X| + |Y| <= 3 * 128 NP)
    __device__ __forceinline__ int get(int x, int p, int y, int i) const {
        const int X = v[i >> 2][x][p][0][i & 3], Y = v[i >> 2][x][p][1][i & 3];
        return (y ? X - Y : X + Y) >> 1;
    }
    // (X, Y) of plane 0, channel_a x: X + Y = 2 S(x, in), X - Y = 2 S(x, major)
    __device__ __forceinline__ int2 raw(int x, int i) const {
        return make_int2(v[i >> 2][x][0][0][i & 3], v[i >> 2][x][0][1][i & 3]);
    }
    static __device__ __forceinline__ uint32_t a_local(int i, uint32_t wave, uint32_t lane) {
        return 16 * (wave & 3) + 4 * (lane >> 4) + (i & 3);
    }
    static __device__ __forceinline__ uint32_t b_local(int i, uint32_t wave, uint32_t lane) {
        return 16 * (NB * (wave >> 2) + (i >> 2)) + (lane & 15);
    }
};

// The same 12 products for 64 sequences with v_mfma_i32_16x16x64_i8: the
// wave's 16 a sites (ca) against the tile's 64 b sites in four 16-column
// blocks (cb[n]).  Lane group g = lane >> 4 carries sequences 16g..16g+15 in
// A, B and the digits alike, so the products pair the same sequence whatever
// the k order inside the instruction.  48 MFMAs of 16 cycles = the 24 of 32 of
// two 32x32 stages; each A operand (digit x channel) feeds 8 MFMAs, so it
// takes 56 v_perm per 48 MFMAs (64 with a 32x32 wave tile).
template <int NPL, int NB>
__device__ __forceinline__ void mfma_block_sel16(v4i (&acc)[NB][2][NPL][2], v4i ca, const v4i (&cb)[NB],
                                                 const v4i (&dp)[NPL]) {
    constexpr unsigned kOnes = 0x01010101u;
    v4i b_in[NB], b_maj[NB];
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            // 0/1/2-coded B: the raw bytes (minor + 2 major) and the minor bit, one v_and per dword
            b_in[n][e] = cb[n][e];
            b_maj[n][e] = cb[n][e] & (int)kOnes;
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
        for (int n = 0; n < NB; ++n) {
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
template <int NPL, int NB>
__device__ __forceinline__ void zero_acc(Acc16<NPL, NB> &acc) {
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int p = 0; p < NPL; ++p)
#pragma unroll
                for (int y = 0; y < 2; ++y)
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc.v[n][x][p][y][e] = 0;
}

// What a pair-kernel launch does with each tile's sums (pair_eval /
// tile_epilogue):
//   kModeDense     every pair's stats to dense matrices (tests)
//   kModeAll       reference epilogue for every valid pair, compaction
//   kModePrefilter the same, skipping pairs that r2_bound_skip proves cannot
//                  pass (exact sums, R = 0; threshold > 0)
//   kModeScreen    one weight-digit plane only (the top one): every valid
//                  pair's r2 is bounded with the plane's residual bound R; a
//                  tile with any pair the bound cannot reject is appended to
//                  the candidate list (recomputed with every plane by the
//                  kModePrefilter launch), the others write their zero counts
//   kModeRefPairs  every valid pair r2_bound_skip cannot reject with the
//                  reference's rounding (plus any omitted planes) as residual (sc.R) is
//                  staged as a candidate row, and each tile's slice of them
//                  recorded (sc.cand_list, sc.cand_count): ref_rows_kernel
//                  (pair_valu.hip) then sums those pairs in lib.rs's order and
//                  keeps the ones that pass
enum : int { kModeDense = 0, kModeAll = 1, kModePrefilter = 2, kModeScreen = 3, kModeRefPairs = 4 };

// the one-plane screen's doubled sums |2S| <= 256 NP stay exact in f32 up to here
constexpr uint32_t kScrF32MaxNP = 16384;

// per-launch screen/candidate arguments
struct ScreenArgs {
    double R;               // kModeScreen: residual bound in top-digit units
    float Rf;               // R rounded up to f32
    float E, mloc;          // f32 == 2: screen_consts of the launch (doubled sums)
    int f32;                // kModeScreen: per-pair test in f32 (nonneg, NP <= kScreenF32MaxNP)
    int nonneg;             // all weights >= 0 (exact 2x2 cells are >= 0)
    uint32_t *cand_list;    // kModeScreen: candidate tiles (packed ta << 16 | tb)
    unsigned *cand_count;   // kModeScreen: appended to; candidate launch: tile count
    uint32_t *cand_bits;    // kModeScreen: per list entry, its 16x16 sub-blocks holding a candidate pair
    unsigned *cand_work;    // the candidate launch's work counter (kModeScreen: workgroup 0 zeroes it)
    unsigned *cand_buckets; // the list's 16 bucket counts (cand_entry; the list and bits: 16 cand_cap each)
    uint32_t cand_cap;
    // kModeScreen for the f32 reference-order candidate launch: list entries
    // are items of a candidate tile's 16-row blocks that hold candidate
    // sub-blocks, packed in row order up to four sub-blocks per item (bits:
    // the item's sub-blocks; bucket 4 - count, cand_cap = 4 tiles), each
    // computed by one workgroup, one sub-block per wave (pair_valu_kernel NS
    // = 1), which owns its row blocks' segments; the tile's row blocks
    // without a candidate get their zero counts here
    int rb_items;
    ScanArgs scan;          // screen and candidate launches: the fused chunk scan (scan_tail)
    // the fp6 screen: a workgroup that finds more than bail candidate tiles
    // listed gives the pass up (kAbandonBit) instead of computing its tile
    // (0: never)
    uint32_t bail;
    // the fp6 screen's sample run (capi.hip fp6_probe): workgroup i screens
    // list entry i * probe_stride + i % probe_stride and only counts, into
    // probe[0] its tiles that hold a pair the bound cannot reject and into
    // probe[1] its tiles (no candidate list, counts or progress written)
    unsigned *probe;
    uint32_t probe_stride;
};

// Reference epilogue of one pair from its exact sums (fixed-point units):
// the optional prefilter, then lib.rs:482-520 in f32.  Returns true when the
// pair passes (valid and r2 > thr, lib.rs:660); d/dp/r2 are written when the
// f32 epilogue ran (always for kModeDense).
template <int MODE>
__device__ __forceinline__ bool pair_eval(double T, double SA, double SB, double SAB, bool valid, float thr,
                                          double scale, bool nonneg, double R, float &d, float &dp, float &r2) {
    if constexpr (MODE != kModeDense) {
        if (!valid) return false;
        // the f32 epilogue below provably gives r2 <= thr (pair_common.hpp)
        if constexpr (MODE == kModePrefilter)
            if (r2_bound_skip(T, SA, SB, SAB, 0.0, thr, nonneg)) return false;
        // ... or, with the reference's rounding as the sums' residual R, the
        // reference's own f32 sums cannot give r2 > thr either; the others are
        // candidates (their values come from ref_rows_kernel)
        if constexpr (MODE == kModeRefPairs) {
            d = dp = r2 = 0.0f;
            return !r2_bound_skip(T, SA, SB, SAB, R, thr, nonneg);
        }
    }
    ld_epilogue((float)(T * scale), (float)(SA * scale), (float)(SB * scale), (float)(SAB * scale), d, dp, r2);
    return valid && r2 > thr;
}

// The screen's verdict on one tile, by its 256 threads (tid: the thread's
// index in the tile's group): bits = the 16x16 sub-blocks that may hold a
// passing pair (nonzero: a candidate, listed; zero: rejected, finished here)
__device__ __forceinline__ void screen_verdict(uint32_t bits, uint32_t ta, uint32_t tb, uint32_t tid,
                                               uint32_t n_chunk_rows, const OrderArgs &o, const ScreenArgs &sc) {
    const uint32_t a0 = ta * kTile;
    if (bits) {
    if (tid == 0) {
        const uint32_t nb = (uint32_t)__popc(bits);  // nb >= 1
        atomicAdd(sc.cand_count, 1u);
        atomicAdd(sc.cand_count + 1, nb);  // sub-blocks to compute (stats)
        // (a list entry: a slot of its bucket; none once the pass is
        // given up, whose mark sits in bucket 0's count)
        auto slot = [&](uint32_t bucket) -> uint32_t {
            const uint32_t k = atomicAdd(&sc.cand_buckets[bucket], 1u);
            return (k & kAbandonBit) || k >= sc.cand_cap ? ~0u : bucket * sc.cand_cap + k;
        };
        if (!sc.rb_items) {
            const uint32_t e = slot(16u - nb);
            if (e != ~0u) {
                sc.cand_list[e] = (ta << 16) | tb;
                sc.cand_bits[e] = bits;
            }
        } else {
            // the tile's 16-row blocks in order, packed greedily into
            // items of at most four computed sub-blocks (one per wave)
            uint32_t empty = 0, cur = 0, cur_k = 0;
            auto emit = [&]() {
                const uint32_t e = slot(4u - cur_k);
                if (e != ~0u) {
                    sc.cand_list[e] = (ta << 16) | tb;
                    sc.cand_bits[e] = cur;
                }
            };
            for (uint32_t q = 0; q < 4; ++q) {
                const uint32_t rb = (bits >> (4 * q)) & 0xFu, k = (uint32_t)__popc(rb);
                if (!k) {
                    ++empty;
                    continue;
                }
                if (cur_k + k > 4) {
                    emit();
                    cur = cur_k = 0;
                }
                cur |= rb << (4 * q);
                cur_k += k;
            }
            if (cur_k) emit();
            if (empty) tile_done(o, ta, tb, n_chunk_rows, empty);  // (quarters: no candidate there)
        }
    }
    if (sc.rb_items && tid < kTile && !((bits >> (4 * (tid >> 4))) & 0xFu))
        o.seg_cnt[(size_t)(a0 + tid) * o.T + tb] = 0;  // a row block without a candidate: no rows
    } else {
        if (tid < kTile) o.seg_cnt[(size_t)(a0 + tid) * o.T + tb] = 0;
        if (tid == 0) tile_done(o, ta, tb, n_chunk_rows);  // rejected: finished here
    }
}

// Epilogue of one 64x64 tile.  The lane holds 16 (a, b) pairs (Acc::a_local,
// b_local).  kModeDense writes every pair's stats (tests); kModeAll and
// kModePrefilter compact passing pairs through the tile's 64x64 pass-bit
// matrix in LDS into staging, with per-(a, b-tile) segment counts and offsets
// for order.hip; kModeScreen only decides whether the tile is a candidate.
//
// sum(x, y, i) returns the lane's i-th pair's sum over channel_a x (0 = in,
// 1 = major) and channel_b y as an exact integer in f64: in fixed-point units
// (S = sum_p 2^(8p) acc_p), or for kModeScreen in units of the screened plane.
template <int MODE, class Acc, class SumFn>
__device__ __forceinline__ void tile_epilogue(const SumFn &sum, const Acc &acc, uint32_t ta, uint32_t tb, uint32_t tid,
                                              uint64_t okA, uint64_t okB, uint32_t L, uint32_t n_chunk_rows,
                                              float thr, int shift, const OrderArgs &o, const DenseArgs &dn,
                                              const ScreenArgs &sc, unsigned long long *sBits, uint32_t *sRowBase) {
    const uint32_t wave = tid >> 6, lane = tid & 63;
    const uint32_t a0 = ta * kTile, b0 = tb * kTile;
    const double scale = ldexp(1.0, -shift);
    if constexpr (MODE == kModeScreen) {
        // sums in units of the screened digit plane, within R of the exact
        // sums scaled to that unit (cells: sum_c |e_c| <= R)
        // the f32 tests need one plane's sums (<= 128 NP); two planes
        // (Acc::kPlanes == 2, the low-threshold screen) always take r2_bound_skip
        const bool f32x2 = Acc::kPlanes == 1 && sc.f32 == 2, f32x1 = Acc::kPlanes == 1 && sc.f32 == 1;
        const float thr_c = thr * (1.0f - 0x1p-7f), R2 = 2.0f * sc.Rf;
        // f32x2: the f32 bound as a violation margin, branch-free, from the
        // doubled sums straight from the X/Y accumulators (raw(x, i) = {2T,
        // 2SB} / {2SA, 2SAB}: exact integers <= 256 NP <= 2^22); E and 2^-12
        // Tb fixed per launch from Tg = 2 sum |top digits| >= every doubled T
        // (screen_consts); the terms straight from X/Y (r2_screen_terms_xy);
        // each term's f32 bits as an int: the maximum is > 0 iff some term is
        // > 0 (finite terms: integer sums <= 2^22)
        auto margin = [&](int i) {
            const auto p0 = acc.raw(0, i), p1 = acc.raw(1, i);  // (X, Y) of channel_a in, major
            float t2;
            const float t1 = r2_screen_terms_xy((float)p0.x, (float)p0.y, (float)p1.x, (float)p1.y, R2, thr_c, sc.E,
                                                sc.mloc, t2);
            return max(__float_as_int(t1), __float_as_int(t2));
        };
        auto valid_pair = [&](int i) {
            const uint32_t a_local = Acc::a_local(i, wave, lane), b_local = Acc::b_local(i, wave, lane);
            return ((okB >> b_local) & 1) && a0 + a_local < b0 + b_local && ((okA >> a_local) & 1);
        };
        // pair i may pass (valid, and the bound does not reject it)
        auto pair_cand = [&](int i) -> bool {
            if (!valid_pair(i)) return false;
            if (f32x2) return margin(i) > 0;
            // the f32 test decides almost every pair; the f64 one the rest
            if (f32x1 && r2_screen_skip_f32((float)sum(0, 0, i), (float)sum(1, 0, i), (float)sum(0, 1, i),
                                            (float)sum(1, 1, i), sc.Rf, thr))
                return false;
            return !r2_bound_skip(sum(0, 0, i), sum(1, 0, i), sum(0, 1, i), sum(1, 1, i), sc.R, thr,
                                  f32x1 || sc.nonneg != 0);
        };
        bool cand = false;
        if (f32x2 && okA == ~0ull && okB == ~0ull && ta != tb) {
            // every pair valid (the tile touches neither the diagonal nor a
            // filtered/padding site)
            int worst = -1;
#pragma unroll
            for (int i = 0; i < Acc::kPairs; ++i) worst = max(worst, margin(i));
            cand = worst > 0;
        } else {
#pragma unroll
            for (int i = 0; i < Acc::kPairs; ++i)
                if (!cand) cand = pair_cand(i);
        }
        unsigned long long *sMask = sBits;  // (no compaction in this mode)
        if (tid == 0) *sMask = 0ull;
        if (__syncthreads_or(cand)) {
            // which 16x16 sub-blocks hold a pair that may pass: the candidate
            // launch computes only those (the others' pairs provably fail)
            unsigned m = 0;
#pragma unroll
            for (int i = 0; i < Acc::kPairs; ++i)
                if (pair_cand(i)) m |= 1u << sub_block<Acc>(i, wave, lane);
            if (m) atomicOr(sMask, (unsigned long long)m);
            __syncthreads();
            screen_verdict((uint32_t)*sMask, ta, tb, tid, n_chunk_rows, o, sc);
        } else {
            screen_verdict(0u, ta, tb, tid, n_chunk_rows, o, sc);
        }
        return;
    }
    float res[Acc::kPairs][3];
    uint32_t pass = 0;
#pragma unroll
    for (int i = 0; i < Acc::kPairs; ++i) {
        const uint32_t a_local = Acc::a_local(i, wave, lane);
        const uint32_t b_local = Acc::b_local(i, wave, lane);
        const uint32_t a = a0 + a_local, b = b0 + b_local;
        const bool valid = ((okB >> b_local) & 1) && a < b && ((okA >> a_local) & 1);
        float d = 0.f, dp = 0.f, r2 = 0.f;
        const bool ok =
            pair_eval<MODE>(sum(0, 0, i), sum(1, 0, i), sum(0, 1, i), sum(1, 1, i), valid, thr, scale, sc.nonneg != 0,
                            sc.R, d, dp, r2);
        res[i][0] = d;
        res[i][1] = dp;
        res[i][2] = r2;
        if constexpr (MODE == kModeDense) {
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
    if constexpr (MODE == kModeDense) return;

    // ---- compaction: a 64x64 pass-bit matrix in LDS, rows in b order ----------
    // A tile with no passing pair (every tile at the bench threshold on random
    // data) writes only its 64 zero counts (seg_off is read only where
    // seg_cnt > 0).  One barrier decides it.
    if (!__syncthreads_or(pass != 0)) {
        if (tid < kTile) o.seg_cnt[(size_t)(a0 + tid) * o.T + tb] = 0;
        if (tid == 0) tile_done(o, ta, tb, n_chunk_rows);
        return;
    }
    if (tid < kTile) sBits[tid] = 0ull;
    __syncthreads();
    if (pass) {
#pragma unroll
        for (int i = 0; i < Acc::kPairs; ++i)
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
        if (rr == 63 && total) {
            base = atomicAdd(o.cursor, (unsigned long long)total);
            if constexpr (MODE == kModeRefPairs) {  // the tile's slice of candidate rows
                const unsigned k = atomicAdd(sc.cand_count, 1u);
                sc.cand_list[3 * k] = (uint32_t)base;
                sc.cand_list[3 * k + 1] = total;
                sc.cand_list[3 * k + 2] = (ta << 16) | tb;
            }
        }
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
        for (int i = 0; i < Acc::kPairs; ++i) {
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
    // (kModeRefPairs: the tile's candidates are summed and compacted by
    // ref_sums / ref_compact, which reports the tile done after that)
    if (MODE != kModeRefPairs && tid == 0) tile_done(o, ta, tb, n_chunk_rows);
}

// LDS-streaming kernel over fragment-major, selector-coded codes, one 64x64
// tile per workgroup; with LOOP (the candidate launch after a screen, whose
// list length tile_count is only known on the device) workgroup i computes
// tiles i, i + gridDim.x, ... (a separate instantiation: the loop costs
// registers the one-tile kernel does not have to give up).  (An
// XCD-contiguous block->tile remap measured no gain: the 41 MB code copy of
// BASELINE config 4 is served from L2/MALL either way.)
template <int MODE, int NPL, bool LOOP>
__global__ __launch_bounds__(64 * GroupShape<NPL>::kWaves, GroupShape<NPL>::kWgPerCu) void pair_mfma_kernel(
    const uint8_t *__restrict__ frag, const uint8_t *__restrict__ frag_b, const int8_t *__restrict__ planes,
    const uint64_t *__restrict__ ok_bits, const uint32_t *__restrict__ tiles, uint32_t n_tiles,
    const unsigned *tile_count, uint32_t L, uint32_t NP, uint32_t n_chunk_rows, float thr, int shift,
    uint32_t plane_idx, OrderArgs o, DenseArgs dn, ScreenArgs sc) {
    constexpr int KG = GroupShape<NPL>::kStages, KGB = GroupShape<NPL>::kBytes;
    constexpr int WAVES = GroupShape<NPL>::kWaves, NB = GroupShape<NPL>::kNB;
    __shared__ __attribute__((aligned(16))) uint8_t smem[2 * KGB];  // operand groups (DMA targets)
    __shared__ unsigned long long sBits[kTile];                              // compaction (never a DMA target)
    __shared__ uint32_t sRowBase[kTile];

    auto compute_tile = [&](uint32_t tile, uint32_t tid) {
        const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
        const uint32_t NKB = NP / 32;
        const uint32_t n_groups = (NKB + KG - 1) / KG;
        const uint32_t ta = tile >> 16, tb = tile & 0xFFFFu;

        // this wave's 1 KB code block per stage: A0/A1 (a sites, selector-coded
        // copy), B0/B1 (b sites, 0/1/2-coded copy); with eight waves, waves w
        // and w + 4 copy the same block of alternate stages
        const uint32_t wb = wave & 3;
        const uint32_t g = wb < 2 ? 2 * ta + wb : 2 * tb + (wb - 2);
        const uint8_t *src = (wb < 2 ? frag : frag_b) + (size_t)g * NKB * 1024;  // wave-uniform
        const int8_t *digf = planes + digf_offset(NP);
        const uint32_t smem_lds = lds_addr(smem);
        auto issue = [&](uint32_t grp, uint32_t buf) {
            const uint32_t gb = smem_lds + buf * KGB;
            const uint32_t kb0 = grp * KG;
            const uint8_t *base = src + (size_t)kb0 * 1024;  // wave-uniform (SGPR base, lane offset in a VGPR)
            const uint32_t lane16 = lane * 16;
#pragma unroll
            for (int st = 0; st < KG; ++st)
                if ((WAVES == 4 || (uint32_t)(st & 1) == (wave >> 2)) && kb0 + st < NKB)
                    glds16_s(base + st * 1024, lane16, gb + st * kStageCodes + wb * 1024);
            // digit records of the group's stages (128 B each, contiguous from
            // digf_stage(kb0)): one 1 KB full-wave copy (allocation padded past
            // the last group)
            if (wave == 0) glds16_s(digf + digf_stage(kb0), lane16, gb + KG * kStageCodes);
        };

        issue(0, 0);
        const uint64_t okA = ok_bits[ta], okB = ok_bits[tb];
        // lane group g = lane >> 4 reads stage 2s + (g >> 1), half g & 1, of each
        // 64-sequence step (the 32-stage fragment layout, re-addressed): a sites
        // 16w.. = rows 16(w & 1).. of 32-site block w >> 1 (w = wave & 3); b
        // block nb = rows 16(nb & 1).. of B block nb >> 1
        const uint32_t g4 = lane >> 4, so = g4 >> 1, hh = g4 & 1;
        const uint32_t lrow = so * kStageCodes + (32 * hh + (lane & 15)) * 16;
        const uint32_t offA = lrow + (wb >> 1) * 1024 + (wb & 1) * 256;
        const uint32_t offB = lrow + 2048 + (WAVES == 8 ? (wave >> 2) * 1024 : 0);  // + (n >> 1) * 1024 + (n & 1) * 256
        const uint32_t offD = KG * kStageCodes + so * kDigStage + hh * 16;
        // the active planes' 32-byte rows of a stage's digit record (NPL 3 is
        // always planes 0-2 and NPL 4 all four: compile-time offsets, kept as
        // immediates)
        uint32_t offP[NPL];
#pragma unroll
        for (int j = 0; j < NPL; ++j) offP[j] = offD + 32 * (NPL >= 3 ? j : ((plane_idx >> (2 * j)) & 3));

        Acc16<NPL, NB> acc;
        zero_acc(acc);
        uint32_t buf = 0;
        for (uint32_t grp = 0; grp < n_groups; ++grp) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's copies of this group landed
            __builtin_amdgcn_s_barrier();                     // ... and every other wave's; the other buffer is free
            asm volatile("" ::: "memory");
            if (grp + 1 < n_groups) issue(grp + 1, buf ^ 1);
            const uint8_t *gb = smem + buf * KGB;
            const uint32_t n_st = min((uint32_t)KG, NKB - grp * KG);
            for (uint32_t st = 0; st < n_st; st += 2) {  // n_st is even: NP is a multiple of 64
                const uint8_t *sc_ = gb + st * kStageCodes;
                const uint8_t *sd = gb + st * kDigStage;
                const v4i ca = *reinterpret_cast<const v4i *>(sc_ + offA);
                v4i cb[NB];
#pragma unroll
                for (int n = 0; n < NB; ++n)
                    cb[n] = *reinterpret_cast<const v4i *>(sc_ + offB + (n >> 1) * 1024 + (n & 1) * 256);
                v4i dp[NPL];
#pragma unroll
                for (int j = 0; j < NPL; ++j) dp[j] = *reinterpret_cast<const v4i *>(sd + offP[j]);
                mfma_block_sel16<NPL, NB>(acc.v, ca, cb, dp);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads of this buffer done before the next barrier
            buf ^= 1;
        }
        const bool narrow = NP <= 65024u;
        auto sum = [&](int x, int y, int i) {
            if constexpr (MODE == kModeScreen && NPL == 1) {
                return acc.get(x, 0, y, i);  // units of the screened plane (int, exact)
            } else if constexpr (MODE == kModeScreen) {
                // two-plane screen (planes lo, lo + 1 = plane_idx's two slots):
                // units of plane lo, |S| <= 2^15 * 128 NP, exact in f64
                static_assert(NPL == 2, "the screen runs on one or two planes");
                return fma(256.0, (double)acc.get(x, 1, y, i), (double)acc.get(x, 0, y, i));
            } else if constexpr (NPL >= 3) {
                // S = sum_p 2^(8p) acc_p, integers below 2^53, exact in f64.
                // |acc_p| <= 128 NP, so acc_1 + 2^8 acc_2 (and acc_2 + 2^8 acc_3)
                // is exact in int32 while 32896 NP < 2^31 (NP <= 65024; the
                // host keeps 4 planes within that).
                if constexpr (NPL == 4) {
                    if (narrow) {
                        const int h23 = acc.get(x, 2, y, i) + acc.get(x, 3, y, i) * 256;
                        const int lo = acc.get(x, 0, y, i) + acc.get(x, 1, y, i) * 256;
                        return (double)fma(65536.0, (double)h23, (double)lo);
                    }
                    return fma(16777216.0, (double)acc.get(x, 3, y, i),
                               fma(65536.0, (double)acc.get(x, 2, y, i),
                                   fma(256.0, (double)acc.get(x, 1, y, i), (double)acc.get(x, 0, y, i))));
                } else {
                    if (narrow) {
                        const int h12 = acc.get(x, 1, y, i) + acc.get(x, 2, y, i) * 256;
                        return fma(256.0, (double)h12, (double)acc.get(x, 0, y, i));
                    }
                    return fma(65536.0, (double)acc.get(x, 2, y, i),
                               fma(256.0, (double)acc.get(x, 1, y, i), (double)acc.get(x, 0, y, i)));
                }
            } else {
                // all-zero planes skipped: sum_j 2^(8 idx_j) acc_j, exact
                double v = 0.0;
#pragma unroll
                for (int j = 0; j < NPL; ++j)
                    v = fma((double)(1u << (8 * ((plane_idx >> (2 * j)) & 3))), (double)acc.get(x, j, y, i), v);
                return v;
            }
        };
        tile_epilogue<MODE, Acc16<NPL, NB>>(sum, acc, ta, tb, tid, okA, okB, L, n_chunk_rows, thr, shift, o, dn, sc, sBits,
                                            sRowBase);
    };
    if constexpr (!LOOP) {
        if constexpr (MODE == kModeScreen || MODE == kModeRefPairs)
            if (blockIdx.x == 0 && threadIdx.x == 0) *sc.cand_work = 0u;  // for the launch after it
        const uint32_t tile = tiles[blockIdx.x];
        if (tile != kNoTile) compute_tile(tile, threadIdx.x);  // kNoTile: padding of an XCD-ordered list
    } else {
        // the first tile by workgroup id, the next ones from the work counter
        __shared__ uint32_t s_next, s_pre[17];
        const uint32_t nt = (*tile_count & kAbandonBit) ? 0u : *tile_count;
        if (blockIdx.x < nt) cand_prefix(sc.cand_buckets, s_pre);  // (a workgroup without a tile skips it)
        for (uint32_t bi = blockIdx.x; bi < nt;) {
            // the thread id laundered per tile: nothing lane-derived is hoisted
            // out of the loop and held live across the epilogue
            uint32_t tid = threadIdx.x;
            asm volatile("" : "+v"(tid));
            // (the entry, then its tile, checked before anything is read through them)
            const uint32_t e = cand_entry_checked(o, s_pre, sc.cand_cap, bi);
            const uint32_t tile = e != ~0u ? tiles[e] : kNoTile;
            if (tile_in_range(tile, L))
                compute_tile(tile, tid);
            else if (e != ~0u && threadIdx.x == 0)
                report_guard(o, kGuardTile);
            if (threadIdx.x == 0) s_next = gridDim.x + atomicAdd(sc.cand_work, 1u);
            __syncthreads();  // (also: the next tile's first DMA reuses buffer 0 and the compaction state)
            bi = s_next;
            __syncthreads();
        }
        scan_tail(sc.scan, nt);
    }
}

// ---- fp6 screen (block-scaled MFMA, twice the i8 rate) ----------------------
//
// The one-plane screen's sums from v_mfma_scale_f32_16x16x128_f8f6f4 with fp6
// (e2m3) operands on both sides, unit block scales: 128 sequences per
// instruction at the cycles of the i8 kernel's 64.  Every weight is rounded
// to its nearest e2m3 value at a common scale S (w6_k = fp6(S w_k), a multiple
// of 1/8 in [0, 7.5]); A = w6 where the a site's symbol is major or minor
// ("in", lib.rs:435) or major (lib.rs:430-432), two channels.  B holds one
// 6-bit code per b symbol, 0 (neither), 8 (major) or 16 (minor), and each B
// register is multiplied twice: read as e2m3 (blgp 2) the codes are 0 / 1.0 /
// 2.0, read as e3m2 (blgp 3) 0 / 0.5 / 2.0 (tools/probes/fp6_dual_probe.hip)
// — two independent channels from the same bytes, with no mask instruction.
// Per pair the four accumulators (channel_a in / major x reading F / G) are
//   F0 = 2T - SB, G0 = 2T - 1.5 SB, F1 = 2SA - SAB, G1 = 2SA - 1.5 SAB
// (T, SA, SB, SAB: lib.rs:441-444's sums of the rounded weights).  Products
// are exact and every sum is a multiple of 1/16 below 2^19, so the f32 MFMA
// sums are exact, and so is every marginal the per-pair test forms from them
// (r2_screen_terms_fg; R is put on the same grid): the screen's f32 bound
// holds with R = sum_k |S w_k - w6_k| plus the reference's rounding, in the
// same units (capi.hip fp6_prepare).  Operands come pre-packed from memory,
// per 64-site tile and 128-sequence block kb one contiguous stage image:
//   a6 [tile][kb][16-site block][channel in, major][1536 B] (12 KB): lane l =
//      site l & 15 of the block, sequences 32 (l >> 4) + j at bits 6j of six
//      dwords, dwords 0-3 at 16 l, dwords 4-5 at 1024 + 8 l (one ds_read_b128
//      and one ds_read_b64 fill the operand registers in place)
//   b6 [tile][kb][16-site block][1536 B]: the b codes, same packing (6 KB)
// One 64x64 tile per 4-wave workgroup, four per CU; per 128 sequences the
// waves LDS-DMA the row tile's A image and the column tile's B image (18 1-KB
// pieces) into a double-buffered 18 KB stage; wave w computes a rows 16w..
// against the four column blocks (16 MFMAs per stage), then the screen
// epilogue.
// B operand: the b codes as fp4 (e2m1) nibbles of minor + 2 major (1.0 /
// 2.0; 16 B per lane and block), the minor channel by one mask per dword (raw
// & 0x2222...), accumulators X / Y (r2_screen_terms_xy2).  (Round 5 measured
// the alternatives and removed them: 6-bit codes read twice as e2m3 / e3m2,
// slower per MFMA and 1.5x the B bytes; a minor-bit plane copied into LDS
// beside B, a larger stage; DESIGN.md Appendix A.)
constexpr int kF6ABytes = 3072;                         // per 16-site block: A, two channels
constexpr int kF6BBytes = 1024;                         // ... and B (fp4 codes)
constexpr int kF6AStage = 4 * kF6ABytes;                // a tile's A image per 128 sequences
constexpr int kF6BStage = 4 * kF6BBytes;                // ... and B image
constexpr int kF6Stage = kF6AStage + kF6BStage;
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

size_t fp6_a_bytes(size_t LP, size_t NP) { return LP / 64 * ((NP + 127) / 128) * kF6AStage; }
size_t fp6_b_bytes(size_t LP, size_t NP) { return LP / 64 * ((NP + 127) / 128) * kF6BStage; }

// one thread per (64-site tile, 128-sequence block, 16-site block, lane)
__global__ __launch_bounds__(256) void frag6_kernel(const uint8_t *__restrict__ codes, const uint8_t *__restrict__ w6,
                                                     uint32_t LP, uint32_t NP, uint8_t *__restrict__ a6,
                                                     uint8_t *__restrict__ b6) {
    const uint32_t NK = (NP + 127) / 128;
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (size_t)LP / 16 * NK * 64) return;
    const uint32_t lane = idx & 63, blk = (idx >> 6) & 3;
    const size_t tk = idx >> 8, tile = tk / NK;  // tk = tile * NK + kb
    const uint32_t kb = (uint32_t)(tk % NK);
    const uint8_t *row = codes + (tile * 64 + blk * 16 + (lane & 15)) * (size_t)NP;
    const uint32_t k0 = 128 * kb + 32 * (lane >> 4);
    uint32_t ai[6] = {0, 0, 0, 0, 0, 0}, am[6] = {0, 0, 0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
    for (uint32_t j = 0; j < 32; ++j) {
        const uint32_t k = k0 + j;
        const uint32_t c = k < NP ? row[k] : 0u, v = k < NP ? w6[k] : 0u;
        const uint32_t vi = (c & kCodeIn) ? v : 0u, vm = (c & kCodeMaj) ? v : 0u;
        const uint32_t bit = 6 * j, d = bit >> 5, o = bit & 31;
        ai[d] |= vi << o;
        am[d] |= vm << o;
        if (o > 26) {
            ai[d + 1] |= vi >> (32 - o);
            am[d + 1] |= vm >> (32 - o);
        }
        // fp4 nibble j: 0, 2 (1.0: minor), 4 (2.0: major)
        b[j >> 3] |= ((c & kCodeIn) ? ((c & kCodeMaj) ? 4u : 2u) : 0u) << (4 * (j & 7));
    }
    uint8_t *pa = a6 + tk * kF6AStage + blk * kF6ABytes, *pm = pa + 1536;
    uint8_t *pb = b6 + tk * kF6BStage + blk * kF6BBytes;
    *reinterpret_cast<uint4 *>(pa + 16 * lane) = make_uint4(ai[0], ai[1], ai[2], ai[3]);
    *reinterpret_cast<uint2 *>(pa + 1024 + 8 * lane) = make_uint2(ai[4], ai[5]);
    *reinterpret_cast<uint4 *>(pm + 16 * lane) = make_uint4(am[0], am[1], am[2], am[3]);
    *reinterpret_cast<uint2 *>(pm + 1024 + 8 * lane) = make_uint2(am[4], am[5]);
    *reinterpret_cast<uint4 *>(pb + 16 * lane) = make_uint4(b[0], b[1], b[2], b[3]);
}

namespace {
// a 16-site block's fp6 operand from its 1536 B LDS image: dwords 0-3, then
// 4-5 (the empty asm keeps the compiler from pairing two blocks' b64 reads
// into one ds_read2, whose four registers would then be copied apart)
__device__ __forceinline__ v8i f6_ld24(const uint8_t *p, uint32_t lane) {
    const uint4 x = *reinterpret_cast<const uint4 *>(p + 16 * lane);
    const uint2 y = *reinterpret_cast<const uint2 *>(p + 1024 + 8 * lane);
    asm volatile("" ::: "memory");
    return v8i{(int)x.x, (int)x.y, (int)x.z, (int)x.w, (int)y.x, (int)y.y, 0, 0};
}
// a 16-site block's B operand (fp4 codes)
__device__ __forceinline__ v8i f6_ldb(const uint8_t *p, uint32_t lane) {
    const uint4 x = *reinterpret_cast<const uint4 *>(p + 16 * lane);
    return v8i{(int)x.x, (int)x.y, (int)x.z, (int)x.w, 0, 0, 0, 0};
}
// one B block's four MFMAs against the wave's A channels (in: ai, major: am):
// acc[channel_a][0 / 1] = X / Y (B raw: minor + 2 major, B's minor bit)
// Zero scale operands: the compiler selects the unscaled
// v_mfma_f32_16x16x128_f8f6f4 (no per-block scales), whose sums equal the
// unit-scaled (E8M0 0x7F) v_mfma_scale form's bit for bit and which issues
// faster: 17.5 / 16.7 / 16.5 against 19.5 / 17.3 / 17.0 cycles per
// instruction at 1 / 2 / 3 waves per SIMD (tools/probes/fp6_unscaled_probe.hip);
// screen C4 -4.1%, 1/8 shard -4.8% (profiles/r06c/).
__device__ __forceinline__ v4f f6_mfma(const v8i &a, const v8i &b, const v4f &c) {
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 2, 4, 0, 0, 0, 0);
}
__device__ __forceinline__ void f6_block_mfma(v4f (&acc)[2][2], const v8i &ai, const v8i &am, const v8i &b) {
    constexpr int kOne = 0;
    constexpr int kMinor = 0x22222222;  // fp4 1.0 (minor) nibbles; 2.0 (major) is 0x4
    const v8i bmin = {b[0] & kMinor, b[1] & kMinor, b[2] & kMinor, b[3] & kMinor, 0, 0, 0, 0};
    acc[0][0] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(ai, b, acc[0][0], 2, 4, 0, kOne, 0, kOne);
    acc[0][1] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(ai, bmin, acc[0][1], 2, 4, 0, kOne, 0, kOne);
    acc[1][0] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(am, b, acc[1][0], 2, 4, 0, kOne, 0, kOne);
    acc[1][1] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(am, bmin, acc[1][1], 2, 4, 0, kOne, 0, kOne);
}
// t1 of pair e of a B block's accumulators, mlo its smallest marginal
__device__ __forceinline__ float f6_terms(const v4f (&acc)[2][2], int e, float R2, float thr_c, float E,
                                          float &mlo) {
    return r2_screen_terms_xy2(acc[0][0][e], acc[0][1][e], acc[1][0][e], acc[1][1][e], R2, thr_c, E, mlo);
}

// The screen epilogue of one wave's 16 rows x 64 columns (acc[n] = b block n),
// the wave being wave wq (0-3) of the 256 threads (ltid) that own tile (ta,
// tb): whether any pair may pass (cand), and its 16x16 sub-block bits
// (blocks: the tile's mask word in LDS, zeroed before).
struct F6Epi {
    uint32_t ta, tb, wq, lane;
    uint64_t okA, okB;
    float R2, thr_c, E, mloc;
    __device__ __forceinline__ bool valid_pair(int i) const {
        const uint32_t al = 16 * wq + 4 * (lane >> 4) + (i & 3), bl = (lane & 15) + 16 * (i >> 2);
        return ((okB >> bl) & 1) && ta * kTile + al < tb * kTile + bl && ((okA >> al) & 1);
    }
    __device__ __forceinline__ bool pair_cand(const v4f (&acc)[4][2][2], int i) const {
        float mlo;
        const float t1 = f6_terms(acc[i >> 2], i & 3, R2, thr_c, E, mlo);
        return valid_pair(i) && (t1 > 0.0f || !(mlo >= mloc));
    }
    // may any of the wave's pairs pass?
    __device__ __forceinline__ bool any(const v4f (&acc)[4][2][2]) const {
        if (okA == ~0ull && okB == ~0ull && ta != tb) {
            // every pair valid (the tile touches neither the diagonal nor a
            // filtered/padding site): branch-free, t1's f32 bits as an int (the
            // maximum is > 0 iff some t1 is > 0; finite terms)
            int worst = -1;
            float mlo_all = INFINITY;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                float mlo;
                worst = max(worst, __float_as_int(f6_terms(acc[i >> 2], i & 3, R2, thr_c, E, mlo)));
                mlo_all = fminf(mlo_all, mlo);
            }
            return worst > 0 || !(mlo_all >= mloc);
        }
        bool cand = false;
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (!cand) cand = pair_cand(acc, i);
        return cand;
    }
    // the wave's sub-block bits (of the tile's 16: 4 (a / 16) + b / 16)
    __device__ __forceinline__ unsigned blocks(const v4f (&acc)[4][2][2]) const {
        unsigned mk = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (pair_cand(acc, i)) mk |= 1u << (4 * wq + (i >> 2));
        return mk;
    }
};
}  // namespace

// one 64x64 tile per 4-wave workgroup, four per CU (tile lists past 2^15
// tile columns, and WLD_OPT_FP6_PAIRS_MIN_TILES's smaller lists)
__global__ __launch_bounds__(256, 4) void pair_fp6_screen_kernel(const uint8_t *__restrict__ a6,
                                                                  const uint8_t *__restrict__ b6,
                                                                  const uint64_t *__restrict__ ok_bits,
                                                                  const uint32_t *__restrict__ tiles, uint32_t n_tiles,
                                                                  uint32_t NK, uint32_t L, uint32_t n_chunk_rows,
                                                                  float thr, OrderArgs o, ScreenArgs sc) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[2 * kF6Stage];
    __shared__ unsigned long long sMask;
    __shared__ uint32_t sBail;
    if (!sc.probe && blockIdx.x == 0 && threadIdx.x == 0) *sc.cand_work = 0u;  // for the launch after it
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t lds = lds_addr(smem), lane16 = lane * 16;
    // (kNoTile: padding of an XCD-ordered list, or past the end of the grid)
    const uint32_t ei = sc.probe ? blockIdx.x * sc.probe_stride + blockIdx.x % sc.probe_stride : blockIdx.x;
    const uint32_t tile = ei < n_tiles ? tiles[ei] : kNoTile;
    if (tile == kNoTile) return;  // (uniform: the whole workgroup)
    const uint32_t ta = tile >> 16, tb = tile & 0xFFFFu;
    const uint8_t *sA = a6 + (size_t)ta * NK * kF6AStage, *sB = b6 + (size_t)tb * NK * kF6BStage;
    // a stage's 1-KB pieces (A image, then the B code blocks): wave w copies w, w + 4, ...
    auto issue = [&](uint32_t kb, uint32_t buf) {
        const uint32_t gb = lds + buf * kF6Stage;
        const uint8_t *a = sA + (size_t)kb * kF6AStage, *b = sB + (size_t)kb * kF6BStage;
#pragma unroll
        for (uint32_t p = wave; p < kF6Stage / 1024; p += 4)
            glds16_s(p < kF6AStage / 1024 ? a + p * 1024 : b + (p - kF6AStage / 1024) * kF6BBytes, lane16, gb + p * 1024);
    };
    issue(0, 0);
    // the give-up test: read by thread 0 while the first stage is in flight,
    // published to the other waves by the first stage barrier (one decision
    // for the workgroup; the LDS write completes before this wave reaches
    // it): 0 go on, 1 give up and mark the set, 2 give up (already marked:
    // the mark is two atomics on one word each; tens of thousands of
    // workgroups repeating them serialise for milliseconds)
    if (tid == 0) {
        uint32_t v = 0;
        if (sc.bail) {
            const unsigned cc = __hip_atomic_load(sc.cand_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            v = cc > sc.bail ? ((cc & kAbandonBit) ? 2u : 1u) : 0u;
        }
        sBail = v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint64_t okA = ok_bits[ta], okB = ok_bits[tb];
    v4f acc[4][2][2];  // [b block n][channel_a in / major][X, Y / F, G]
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y) acc[n][x][y] = v4f{0.0f, 0.0f, 0.0f, 0.0f};
    uint32_t buf = 0;
    for (uint32_t kb = 0; kb < NK; ++kb) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's copies of the stage landed
        __builtin_amdgcn_s_barrier();                     // ... and every other wave's; the other buffer is free
        asm volatile("" ::: "memory");
        if (kb == 0 && sBail) {  // (uniform) give the pass up: drain this wave's copies, leave
            if (tid == 0 && sBail == 1) {
                atomicOr(sc.cand_count, kAbandonBit);
                atomicOr(sc.cand_buckets, kAbandonBit);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            return;
        }
        if (kb + 1 < NK) issue(kb + 1, buf ^ 1);
        const uint8_t *g = smem + buf * kF6Stage;
        const v8i ai = f6_ld24(g + wave * kF6ABytes, lane), am = f6_ld24(g + wave * kF6ABytes + 1536, lane);
#pragma unroll
        for (int n = 0; n < 4; ++n) f6_block_mfma(acc[n], ai, am, f6_ldb(g + kF6AStage + n * kF6BBytes, lane));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads of this buffer done before the next barrier
        buf ^= 1;
    }
    const F6Epi ep{ta, tb, wave, lane, okA, okB, 2.0f * sc.Rf, thr * (1.0f - 0x1p-7f), sc.E, sc.mloc};
    const bool cand = ep.any(acc);
    if (sc.probe) {  // the sample run: count, decide nothing
        const bool any = __syncthreads_or(cand);
        if (tid == 0) {
            if (any) atomicAdd(sc.probe, 1u);
            atomicAdd(sc.probe + 1, 1u);
        }
        return;
    }
    if (tid == 0) sMask = 0ull;
    if (__syncthreads_or(cand)) {
        // which 16x16 sub-blocks hold a pair that may pass: the candidate
        // launch computes only those (the others' pairs provably fail)
        const unsigned mk = ep.blocks(acc);
        if (mk) atomicOr(&sMask, (unsigned long long)mk);
        __syncthreads();
        screen_verdict((uint32_t)sMask, ta, tb, tid, n_chunk_rows, o, sc);
    } else {
        screen_verdict(0u, ta, tb, tid, n_chunk_rows, o, sc);
    }
}

constexpr uint32_t kF6Single = 0x8000u;  // (= tile_order::kSingleEntry)

// Tile pairs: one 4-wave workgroup per entry of the pair list, tiles (ta, tb)
// and (ta, tb + 1) (kF6Single: tile (ta, tb) alone), three workgroups per CU.
// Both tiles' rows are the same 64 sites, so one A image per stage serves
// both: per 128 sequences the workgroup LDS-DMAs A (12 KB) and the two B
// images (2 x 4 KB) into one of two 20-KB stage buffers, each wave five 1-KB
// pieces from bases set once (round 6: C4 -5%, C5 -3%, 1/8 shard -6% against
// selecting each piece's source per stage, profiles/r06b/).  Wide waves: wave
// w computes rows 32 (w & 1) .. + 31 (two 16-row blocks) x 64 columns of tile
// tb + (w >> 1), so each B block is read and masked once for two A row blocks
// (per MFMA 0.31 KB of LDS reads); 128 accumulator registers per lane.  Each
// half decides its own tile; a single entry's second half computes on the
// first B image and decides nothing (it keeps the workgroup's barriers).
// (Measured and removed: eight waves of 16 x 64, three stage buffers, a
// producer/consumer split, register-staged operands (round 5); tile triples
// on six waves, two workgroups per CU (+43%), and the full-tile bound on
// packed f32 (+1%) (round 6); DESIGN.md Appendix A.)
constexpr int kF6PStage = kF6AStage + 2 * kF6BStage;
__global__ __launch_bounds__(256, 3) void pair_fp6_screen2w_kernel(
    const uint8_t *__restrict__ a6, const uint8_t *__restrict__ b6, const uint64_t *__restrict__ ok_bits,
    const uint32_t *__restrict__ pairs, uint32_t n_pairs, uint32_t NK, uint32_t L, uint32_t n_chunk_rows, float thr,
    OrderArgs o, ScreenArgs sc) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[2 * kF6PStage];
    __shared__ unsigned long long sMask[2];
    __shared__ uint32_t sBail, sCand[2];
    if (!sc.probe && blockIdx.x == 0 && threadIdx.x == 0) *sc.cand_work = 0u;  // for the launch after it
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t half = wave >> 1, rp = wave & 1, ltid = tid & 127;
    const uint32_t lds = lds_addr(smem), lane16 = lane * 16;
    const uint32_t ei = sc.probe ? blockIdx.x * sc.probe_stride + blockIdx.x % sc.probe_stride : blockIdx.x;
    const uint32_t entry = ei < n_pairs ? pairs[ei] : kNoTile;
    if (entry == kNoTile) return;  // (uniform: the whole workgroup)
    // a stage's twenty 1-KB pieces (A image 0-11, B image of tb 12-15, of tb
    // + 1 16-19): wave w copies w, w + 4, w + 8 of A and piece w of each B
    // image (a single entry's second image is the first's, which its idle
    // half reads)
    static_assert(kF6AStage == 3 * 4096 && kF6BStage == 4096, "five pieces per wave and stage");
    struct Src {
        const uint8_t *pA, *pB0, *pB1;
    };
    auto src_of = [&](uint32_t e) {
        const uint32_t ta_ = e >> 16, tb0_ = e & 0x7FFFu;
        Src r;
        r.pA = a6 + (size_t)ta_ * NK * kF6AStage + wave * 1024;
        r.pB0 = b6 + (size_t)tb0_ * NK * kF6BStage + wave * 1024;
        r.pB1 = (e & kF6Single) ? r.pB0 : r.pB0 + (size_t)NK * kF6BStage;
        return r;
    };
    auto issue = [&](const Src &sr, uint32_t kb, uint32_t buf) {
        const uint32_t gb = lds + buf * kF6PStage + wave * 1024;
        const uint8_t *a = sr.pA + (size_t)kb * kF6AStage;
        const size_t bo = (size_t)kb * kF6BStage;
        glds16_s(a, lane16, gb);
        glds16_s(a + 4096, lane16, gb + 4096);
        glds16_s(a + 8192, lane16, gb + 8192);
        glds16_s(sr.pB0 + bo, lane16, gb + kF6AStage);
        glds16_s(sr.pB1 + bo, lane16, gb + kF6AStage + kF6BStage);
    };
    const Src cur = src_of(entry);
    issue(cur, 0, 0);
    uint32_t buf = 0;
    {
        const uint32_t ta = entry >> 16, tb0 = entry & 0x7FFFu;
        const bool single = (entry & kF6Single) != 0, idle = single && half;  // (uniform per wave)
        const uint32_t tb = tb0 + (idle ? 0u : half);
        if (tid == 0) {  // the give-up test (as the single-tile kernel)
            uint32_t v = 0;
            if (sc.bail) {
                const unsigned cc = __hip_atomic_load(sc.cand_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                v = cc > sc.bail ? ((cc & kAbandonBit) ? 2u : 1u) : 0u;
            }
            sBail = v;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const uint64_t okA = ok_bits[ta], okB = ok_bits[tb];
        v4f acc[2][4][2][2];  // [row block 2 rp + j][b block n][channel_a][X, Y]
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int n = 0; n < 4; ++n)
#pragma unroll
                for (int x = 0; x < 2; ++x)
#pragma unroll
                    for (int y = 0; y < 2; ++y) acc[j][n][x][y] = v4f{0.0f, 0.0f, 0.0f, 0.0f};
        const uint32_t boff = kF6AStage + (idle ? 0u : half) * kF6BStage;  // this half's B image in a stage
        const uint32_t aoff = 2 * rp * kF6ABytes;                             // this wave's two A row blocks
        for (uint32_t kb = 0; kb < NK; ++kb) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's copies of the stage landed
            __builtin_amdgcn_s_barrier();                     // ... and every other wave's; the other buffer is free
            asm volatile("" ::: "memory");
            if (kb == 0) {
                if (sBail) {  // (uniform) give the pass up: drain this wave's copies, leave
                    if (tid == 0 && sBail == 1) {
                        atomicOr(sc.cand_count, kAbandonBit);
                        atomicOr(sc.cand_buckets, kAbandonBit);
                    }
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    return;
                }
                // (every wave has left the previous entry's epilogue)
                if (tid < 2) sCand[tid] = 0u, sMask[tid] = 0ull;
            }
            if (kb + 1 < NK) issue(cur, kb + 1, buf ^ 1);
            const uint8_t *g = smem + buf * kF6PStage;
            // Two B slots rolled through the stage: block n's raw MFMAs, its
            // minor mask in place, its masked MFMAs, then block n + 2's read
            // into the same slot, in flight under block n + 1's eight MFMAs
            // (round 6: C4 screen -1.6%, LD blocks -2% with the same order in
            // the i8 screen, against reading blocks 2-3 only after blocks
            // 0-1's MFMAs, where the compiler's one register set for them
            // left the read's latency exposed; profiles/r06k/.  Reading row
            // block 0's A and B block 0 first, or the next stage's copies
            // issued after the reads, measured no better: profiles/r06l/)
            const v8i ai0 = f6_ld24(g + aoff, lane), am0 = f6_ld24(g + aoff + 1536, lane);
            const v8i ai1 = f6_ld24(g + aoff + kF6ABytes, lane), am1 = f6_ld24(g + aoff + kF6ABytes + 1536, lane);
            v8i bs[2] = {f6_ldb(g + boff, lane), f6_ldb(g + boff + kF6BBytes, lane)};
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                v8i &b = bs[n & 1];
                constexpr int kMinor = 0x22222222;  // fp4 1.0 (minor) nibbles; 2.0 (major) is 0x4
                acc[0][n][0][0] = f6_mfma(ai0, b, acc[0][n][0][0]);
                acc[0][n][1][0] = f6_mfma(am0, b, acc[0][n][1][0]);
                acc[1][n][0][0] = f6_mfma(ai1, b, acc[1][n][0][0]);
                acc[1][n][1][0] = f6_mfma(am1, b, acc[1][n][1][0]);
                __builtin_amdgcn_sched_barrier(0);
                b = v8i{b[0] & kMinor, b[1] & kMinor, b[2] & kMinor, b[3] & kMinor, 0, 0, 0, 0};
                acc[0][n][0][1] = f6_mfma(ai0, b, acc[0][n][0][1]);
                acc[0][n][1][1] = f6_mfma(am0, b, acc[0][n][1][1]);
                acc[1][n][0][1] = f6_mfma(ai1, b, acc[1][n][0][1]);
                acc[1][n][1][1] = f6_mfma(am1, b, acc[1][n][1][1]);
                __builtin_amdgcn_sched_barrier(0);
                if (n + 2 < 4) b = f6_ldb(g + boff + (n + 2) * kF6BBytes, lane);
                __builtin_amdgcn_sched_barrier(0);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads of this buffer done before the next barrier
            buf ^= 1;
        }
        const F6Epi ep0{ta, tb, 2 * rp, lane, okA, okB, 2.0f * sc.Rf, thr * (1.0f - 0x1p-7f), sc.E, sc.mloc};
        const F6Epi ep1{ta, tb, 2 * rp + 1, lane, okA, okB, 2.0f * sc.Rf, thr * (1.0f - 0x1p-7f), sc.E, sc.mloc};
        const bool cand = !idle && (ep0.any(acc[0]) || ep1.any(acc[1]));
        if (cand) sCand[half] = 1u;  // (benign race: every writer stores 1)
        __syncthreads();
        const bool mine = sCand[half] != 0;  // (uniform per half)
        if (sc.probe) {  // the sample run: count, decide nothing
            if (ltid == 0 && !idle) {
                if (mine) atomicAdd(sc.probe, 1u);
                atomicAdd(sc.probe + 1, 1u);
            }
            return;
        }
        if (mine && !idle) {
            const unsigned mk = ep0.blocks(acc[0]) | ep1.blocks(acc[1]);
            if (mk) atomicOr(&sMask[half], (unsigned long long)mk);
        }
        __syncthreads();
        if (!idle) screen_verdict(mine ? (uint32_t)sMask[half] : 0u, ta, tb, ltid, n_chunk_rows, o, sc);
    }
}

// ---- i8 screen on tile pairs with wide waves (round 6) ----------------------
//
// The one-plane i8 screen (the top weight digit d = d_top)
// where the fp6 rounding is too coarse for the data (linkage blocks, wide
// weight ranges): the tile-pair, wide-wave structure of
// pair_fp6_screen2w_kernel on v_mfma_i32_16x16x64_i8, with the operands
// pre-multiplied once per load (i8_images_build) instead of formed per stage
// by v_perm: per 64-site tile and 64-sequence block kb one stage image
//   A [tile][kb][16-site block][in, major][1 KB]: lane l = site l & 15,
//      byte j = d(k) x in (resp. major) of sequence k = 64 kb + 16 (l >> 4) + j
//      (int8: a digit in [-128, 127] times 0 or 1)                      (8 KB)
//   B [tile][kb][16-site block][1 KB]: the same lanes, byte j = the b code
//      0 (neither), 1 (minor), 2 (major) = minor + 2 major              (4 KB)
// so X = S(A B) and Y = S(A (B & 0x01010101)) are the X / Y sums of the fp6
// screen (X0 = T + SB, Y0 = T - SB, X1 = SA + SAB, Y1 = SA - SAB in
// top-digit units): exact integers below 2^23, so exact in f32, and the same
// epilogue (F6Epi, r2_screen_terms_xy2) decides each tile with R2 = 2R on
// the integer grid.  Per stage (64 sequences) a workgroup LDS-DMAs A (8 KB)
// and two B images (4 KB each); wave w copies four 1-KB pieces and computes
// rows 32 (w & 1) .. + 31 x 64 columns of tile tb + (w >> 1): 32 MFMAs per
// stage, 8 KB of LDS reads, 16 mask instructions.
constexpr int kI8ABytes = 2048;                 // per 16-site block: in, major channels
constexpr int kI8AStage = 4 * kI8ABytes;        // a tile's A image per 64 sequences
constexpr int kI8BStage = 4 * 1024;             // ... and B image
constexpr int kI8PStage = kI8AStage + 2 * kI8BStage;
size_t i8_a_bytes(size_t LP, size_t NP) { return LP / 64 * (NP / 64) * kI8AStage; }
size_t i8_b_bytes(size_t LP, size_t NP) { return LP / 64 * (NP / 64) * kI8BStage; }

// one thread per (64-site tile, 64-sequence block, 16-site block, lane)
__global__ __launch_bounds__(256) void i8img_kernel(const uint8_t *__restrict__ codes, const int8_t *__restrict__ digit,
                                                     uint32_t LP, uint32_t NP, uint8_t *__restrict__ a8,
                                                     uint8_t *__restrict__ b8) {
    const uint32_t NK = NP / 64;
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (size_t)LP / 16 * NK * 64) return;
    const uint32_t lane = idx & 63, blk = (idx >> 6) & 3;
    const size_t tk = idx >> 8, tile = tk / NK;  // tk = tile * NK + kb
    const uint32_t kb = (uint32_t)(tk % NK);
    const uint32_t k0 = 64 * kb + 16 * (lane >> 4);
    const uint4 c4 = *reinterpret_cast<const uint4 *>(codes + (tile * 64 + blk * 16 + (lane & 15)) * (size_t)NP + k0);
    const uint4 d4 = *reinterpret_cast<const uint4 *>(digit + k0);
    const uint32_t c[4] = {c4.x, c4.y, c4.z, c4.w}, d[4] = {d4.x, d4.y, d4.z, d4.w};
    uint32_t ai[4], am[4], b[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint32_t vi = 0, vm = 0, vb = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t cc = (c[q] >> (8 * j)) & 0xFFu, dd = (d[q] >> (8 * j)) & 0xFFu;
            vi |= ((cc & kCodeIn) ? dd : 0u) << (8 * j);
            vm |= ((cc & kCodeMaj) ? dd : 0u) << (8 * j);
            vb |= ((cc & kCodeIn) ? ((cc & kCodeMaj) ? 2u : 1u) : 0u) << (8 * j);
        }
        ai[q] = vi, am[q] = vm, b[q] = vb;
    }
    uint8_t *pa = a8 + tk * kI8AStage + blk * kI8ABytes;
    *reinterpret_cast<uint4 *>(pa + 16 * lane) = make_uint4(ai[0], ai[1], ai[2], ai[3]);
    *reinterpret_cast<uint4 *>(pa + 1024 + 16 * lane) = make_uint4(am[0], am[1], am[2], am[3]);
    *reinterpret_cast<uint4 *>(b8 + tk * kI8BStage + blk * 1024 + 16 * lane) = make_uint4(b[0], b[1], b[2], b[3]);
}

void launch_i8img(const uint8_t *codes, const int8_t *digit, size_t LP, size_t NP, uint8_t *a8, uint8_t *b8,
                  hipStream_t s) {
    const size_t n = LP / 16 * (NP / 64) * 64;
    hipLaunchKernelGGL(i8img_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, codes, digit, (uint32_t)LP,
                       (uint32_t)NP, a8, b8);
}

__global__ __launch_bounds__(256, 3) void pair_i8_screen2w_kernel(
    const uint8_t *__restrict__ a8, const uint8_t *__restrict__ b8, const uint64_t *__restrict__ ok_bits,
    const uint32_t *__restrict__ pairs, uint32_t n_pairs, uint32_t NK, uint32_t L, uint32_t n_chunk_rows, float thr,
    OrderArgs o, ScreenArgs sc) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[2 * kI8PStage];
    __shared__ unsigned long long sMask[2];
    __shared__ uint32_t sCand[2];
    if (blockIdx.x == 0 && threadIdx.x == 0) *sc.cand_work = 0u;  // for the launch after it
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t half = wave >> 1, rp = wave & 1, ltid = tid & 127;
    const uint32_t lds = lds_addr(smem), lane16 = lane * 16;
    const uint32_t entry = blockIdx.x < n_pairs ? pairs[blockIdx.x] : kNoTile;
    if (entry == kNoTile) return;  // (uniform: the whole workgroup)
    const uint32_t ta = entry >> 16, tb0 = entry & 0x7FFFu;
    const bool single = (entry & kF6Single) != 0, idle = single && half;  // (uniform per wave)
    const uint32_t tb = tb0 + (idle ? 0u : half);
    // a stage's sixteen 1-KB pieces (A image 0-7, B image of tb 8-11, of tb + 1
    // 12-15): wave w copies w and w + 4 of A and piece w of each B image
    static_assert(kI8AStage == 2 * 4096 && kI8BStage == 4096, "four pieces per wave and stage");
    const uint8_t *pA = a8 + (size_t)ta * NK * kI8AStage + wave * 1024;
    const uint8_t *pB0 = b8 + (size_t)tb0 * NK * kI8BStage + wave * 1024;
    const uint8_t *pB1 = single ? pB0 : pB0 + (size_t)NK * kI8BStage;
    auto issue = [&](uint32_t kb, uint32_t buf) {
        const uint32_t gb = lds + buf * kI8PStage + wave * 1024;
        const uint8_t *a = pA + (size_t)kb * kI8AStage;
        const size_t bo = (size_t)kb * kI8BStage;
        glds16_s(a, lane16, gb);
        glds16_s(a + 4096, lane16, gb + 4096);
        glds16_s(pB0 + bo, lane16, gb + kI8AStage);
        glds16_s(pB1 + bo, lane16, gb + kI8AStage + kI8BStage);
    };
    issue(0, 0);
    if (tid < 2) sCand[tid] = 0u, sMask[tid] = 0ull;
    const uint64_t okA = ok_bits[ta], okB = ok_bits[tb];
    v4i acc[2][4][2][2];  // [row block 2 rp + j][b block n][channel_a][X, Y]
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y) acc[j][n][x][y] = v4i{0, 0, 0, 0};
    const uint32_t boff = kI8AStage + (idle ? 0u : half) * kI8BStage;  // this half's B image in a stage
    const uint32_t aoff = 2 * rp * kI8ABytes;                             // this wave's two A row blocks
    uint32_t buf = 0;
    for (uint32_t kb = 0; kb < NK; ++kb) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's copies of the stage landed
        __builtin_amdgcn_s_barrier();                     // ... and every other wave's; the other buffer is free
        asm volatile("" ::: "memory");
        if (kb + 1 < NK) issue(kb + 1, buf ^ 1);
        const uint8_t *g = smem + buf * kI8PStage;
        v4i av[2][2];
        auto ldb = [&](int n) { return *reinterpret_cast<const v4i *>(g + boff + n * 1024 + 16 * lane); };
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int x = 0; x < 2; ++x)
                av[j][x] = *reinterpret_cast<const v4i *>(g + aoff + j * kI8ABytes + x * 1024 + 16 * lane);
        // two B slots rolled through the stage, as the fp6 screen (round 6:
        // LD-block screen -2%, profiles/r06k/)
        v4i bs[2] = {ldb(0), ldb(1)};
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            v4i &b = bs[n & 1];
            constexpr int kOnes = 0x01010101;  // the minor bit of each code byte
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int x = 0; x < 2; ++x) acc[j][n][x][0] = mfma_i8_16(av[j][x], b, acc[j][n][x][0]);
            __builtin_amdgcn_sched_barrier(0);
            b = v4i{b[0] & kOnes, b[1] & kOnes, b[2] & kOnes, b[3] & kOnes};
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int x = 0; x < 2; ++x) acc[j][n][x][1] = mfma_i8_16(av[j][x], b, acc[j][n][x][1]);
            __builtin_amdgcn_sched_barrier(0);
            if (n + 2 < 4) b = ldb(n + 2);
            __builtin_amdgcn_sched_barrier(0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads of this buffer done before the next barrier
        buf ^= 1;
    }
    // the integer sums as f32 (exact: |X|, |Y| < 2^23), then the fp6 screen's epilogue
    v4f accf[2][4][2][2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y)
#pragma unroll
                    for (int e = 0; e < 4; ++e) accf[j][n][x][y][e] = (float)acc[j][n][x][y][e];
    const F6Epi ep0{ta, tb, 2 * rp, lane, okA, okB, 2.0f * sc.Rf, thr * (1.0f - 0x1p-7f), sc.E, sc.mloc};
    const F6Epi ep1{ta, tb, 2 * rp + 1, lane, okA, okB, 2.0f * sc.Rf, thr * (1.0f - 0x1p-7f), sc.E, sc.mloc};
    const bool cand = !idle && (ep0.any(accf[0]) || ep1.any(accf[1]));
    if (cand) sCand[half] = 1u;  // (benign race: every writer stores 1)
    __syncthreads();
    const bool mine = sCand[half] != 0;  // (uniform per half)
    if (mine && !idle) {
        const unsigned mk = ep0.blocks(accf[0]) | ep1.blocks(accf[1]);
        if (mk) atomicOr(&sMask[half], (unsigned long long)mk);
    }
    __syncthreads();
    if (!idle) screen_verdict(mine ? (uint32_t)sMask[half] : 0u, ta, tb, ltid, n_chunk_rows, o, sc);
}

void launch_frag6(const uint8_t *codes, const uint8_t *w6, size_t LP, size_t NP, uint8_t *a6, uint8_t *b6,
                  hipStream_t s) {
    const size_t n = LP / 16 * ((NP + 127) / 128) * 64;
    hipLaunchKernelGGL(frag6_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, codes, w6, (uint32_t)LP,
                       (uint32_t)NP, a6, b6);
}

// Site-major variant (one tile per workgroup, codes read straight into
// registers, all three digit planes): the reference for the LDS path's race
// screen (WLD_OPT_MFMA_LAYOUT).
template <int MODE>
__global__ __launch_bounds__(256, 2) void pair_mfma_rows_kernel(const uint8_t *__restrict__ codes,
                                                                 const int8_t *__restrict__ planes,
                                                                 const uint64_t *__restrict__ ok_bits,
                                                                 const uint32_t *__restrict__ tiles, uint32_t L,
                                                                 uint32_t NP, uint32_t n_chunk_rows, float thr,
                                                                 int shift, OrderArgs o, DenseArgs dn, ScreenArgs sc) {
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
    const bool narrow = NP <= 65024u;
    auto sum = [&](int x, int y, int i) -> double {
        if (narrow) {
            const int hi = acc.get(x, 1, y, i) + acc.get(x, 2, y, i) * 256;
            return fma(256.0, (double)hi, (double)acc.get(x, 0, y, i));
        }
        return fma(65536.0, (double)acc.get(x, 2, y, i), fma(256.0, (double)acc.get(x, 1, y, i), (double)acc.get(x, 0, y, i)));
    };
    tile_epilogue<MODE, Acc32<3>>(sum, acc, ta, tb, tid, ok_bits[ta], ok_bits[tb], L, n_chunk_rows, thr, shift, o, dn, sc,
                                  sBits, sRowBase);
}

void launch_mfma_prep(const uint8_t *site_ok, const float *w_pad, size_t L, size_t LP, size_t NP, int shift,
                      int8_t *planes, hipStream_t s) {
    unsigned *stats = reinterpret_cast<unsigned *>(planes + planemask_offset(LP, NP));
    (void)hipMemsetAsync(stats, 0, 64, s);
    hipLaunchKernelGGL(mfma_prep_kernel, dim3((unsigned)((NP + 255) / 256)), dim3(256), 0, s, w_pad, (uint32_t)NP,
                       shift, planes, planes + digf_offset(NP), stats);
    hipLaunchKernelGGL(okbits_kernel, dim3((unsigned)(LP / 64)), dim3(64), 0, s, site_ok, (uint32_t)L,
                       reinterpret_cast<uint64_t *>(planes + okbits_offset(NP)));
}

void launch_frag(const uint8_t *codes, size_t LP, size_t NP, uint8_t *frag, hipStream_t s) {
    const size_t chunks = LP * NP / 16;
    hipLaunchKernelGGL(frag_kernel, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0, s, codes, (uint32_t)LP,
                       (uint32_t)NP, frag);
}

int mfma_weight_stats(const int8_t *wplanes, size_t LP, size_t NP, hipStream_t s, MfmaWeightStats *out) {
    struct {
        unsigned mask, pad;
        unsigned long long resid[3];
        unsigned long long dsum[kMaxPlanes];
    } h{};
    if (hipMemcpyAsync(&h, wplanes + planemask_offset(LP, NP), sizeof(h), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -1;
    out->plane_mask = h.mask & 15;
    out->nonneg = !(h.mask & 0x100);
    for (int t = 0; t < 3; ++t) out->resid[t] = h.resid[t];
    for (int p = 0; p < kMaxPlanes; ++p) out->dsum[p] = h.dsum[p];
    return 0;
}

namespace {
template <int MODE, int NPL, bool LOOP = false>
void launch_lds(const MfmaLaunch &m, const uint64_t *ok_bits, const uint32_t *tiles, uint32_t n_tiles,
                const unsigned *tile_count, uint32_t grid, uint32_t plane_idx, const OrderArgs &o, const DenseArgs &dn,
                const ScreenArgs &sc, hipStream_t s) {
    hipLaunchKernelGGL((pair_mfma_kernel<MODE, NPL, LOOP>), dim3(grid), dim3(64 * GroupShape<NPL>::kWaves), 0, s, m.frag, m.frag_b, m.wplanes,
                       ok_bits, tiles, n_tiles, tile_count, m.L, m.NP, m.n_chunk_rows, m.thr, m.shift, plane_idx, o,
                       dn, sc);
}

template <int MODE, bool LOOP = false>
void launch_lds_planes(uint32_t n_planes, const MfmaLaunch &m, const uint64_t *ok_bits, const uint32_t *tiles,
                       uint32_t n_tiles, const unsigned *tile_count, uint32_t grid, uint32_t plane_idx,
                       const OrderArgs &o, const DenseArgs &dn, const ScreenArgs &sc, hipStream_t s) {
    if (n_planes == 4)
        launch_lds<MODE, 4, LOOP>(m, ok_bits, tiles, n_tiles, tile_count, grid, plane_idx, o, dn, sc, s);
    else if (n_planes == 3)
        launch_lds<MODE, 3, LOOP>(m, ok_bits, tiles, n_tiles, tile_count, grid, plane_idx, o, dn, sc, s);
    else if (n_planes == 2 || LOOP)  // the looping candidate launch follows a screen: >= 2 planes
        launch_lds<MODE, 2, LOOP>(m, ok_bits, tiles, n_tiles, tile_count, grid, plane_idx, o, dn, sc, s);
    else
        launch_lds<MODE, 1, false>(m, ok_bits, tiles, n_tiles, tile_count, grid, plane_idx, o, dn, sc, s);
}
// The candidate launch after a screen: a grid-stride loop over the candidate
// list (length on the device) with every digit plane and the exact
// prefilter, or (WLD_OPT_REF_SUMS) the reference-order f32 kernel.
void launch_candidates(const MfmaLaunch &m, uint32_t n, uint32_t idx, const uint64_t *ok_bits, const OrderArgs &o,
                       const DenseArgs &dn, const ScreenArgs &sc, hipStream_t s) {
    // WLD_OPT_TEST_GUARD: the last bucket's count one past its capacity, so
    // the launch meets an entry outside the buckets (its guard must refuse
    // it); the bucket's slots zeroed first, so the entries below the capacity
    // are tile 0 with no sub-block (refused too) rather than stale data.  The
    // list holds 16 n_tiles entries: buckets 0-15 of n_tiles, or with
    // 16-row items buckets 0-3 of 4 n_tiles
    if (m.test_guard && sc.cand_buckets && m.cand_list && sc.cand_bits && sc.cand_cap) {
        const size_t cap = sc.cand_cap, last = 16 * (size_t)m.n_tiles / cap - 1;
        (void)hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(m.cand_list + last * cap), 0, cap, s);
        (void)hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(sc.cand_bits + last * cap), 0, cap, s);
        (void)hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(sc.cand_buckets + last), (int)(cap + 1), 1, s);
        // ... and the tile count (the exact mode's candidate loop runs to it)
        // past every bucket: its last entry lies beyond their total
        if (m.cand_count)
            (void)hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(m.cand_count), (int)(16 * m.n_tiles + 2), 1, s);
    }
    if (m.ref_valu) {
        ValuLaunch v = *m.ref_valu;
        v.tiles = m.cand_list;
        v.n_tiles = m.n_tiles;
        v.tile_count = m.cand_count;
        v.tile_bits = sc.cand_bits;
        v.tile_work = sc.cand_work;
        v.tile_buckets = sc.cand_buckets;
        v.bucket_cap = sc.cand_cap;
        v.rb_items = sc.rb_items != 0;
        v.scan = sc.scan;
        launch_pair_valu(v, o, nullptr, s);
        return;
    }
    const uint32_t grid = std::min<uint32_t>(m.n_tiles, kCandidateGrid);
    launch_lds_planes<kModePrefilter, true>(n, m, ok_bits, m.cand_list, 0, m.cand_count, grid, idx, o, dn, sc, s);
}
}  // namespace

namespace {
// the fp6 screen's R, E, mloc in its own units (fp6_prepare): R rounded up to
// a multiple of 1/32, so the doubled R2 = 2 R lies on the accumulators' grid
// (1/8 or 1/16: the exact marginals of r2_screen_terms_xy2 / _fg; exact in f32,
// R <= the sum of the fp6 weights < 2^17); Tg bounds every doubled T
void fp6_screen_args(const MfmaLaunch &m, ScreenArgs &sc) {
    sc.R = std::ceil(m.fp6->R * 32.0) / 32.0;
    sc.Rf = (float)sc.R;
    sc.f32 = 2;
    screen_consts(m.fp6->Tg, 2.0f * sc.Rf, sc.E, sc.mloc);
}
// the fp6 screen over the pair list (or the tile list), every entry, or with
// sc.probe every stride-th one
void launch_fp6_screen(const MfmaLaunch &m, const uint64_t *ok_bits, const OrderArgs &o, const ScreenArgs &sc,
                       uint32_t stride, hipStream_t s) {
    if (m.f6_pairs) {
        // (a tile group per workgroup, the XCD-ordered group list)
        hipLaunchKernelGGL(pair_fp6_screen2w_kernel, dim3((m.f6_n_pairs + stride - 1) / stride), dim3(256), 0, s,
                           m.fp6->a6, m.fp6->b6, ok_bits, m.f6_pairs, m.f6_n_pairs, m.fp6->NK, m.L, m.n_chunk_rows,
                           m.thr, o, sc);
    } else {
        // (one tile per workgroup, the XCD-ordered list)
        hipLaunchKernelGGL(pair_fp6_screen_kernel, dim3((m.n_tiles + stride - 1) / stride), dim3(256), 0, s,
                           m.fp6->a6, m.fp6->b6, ok_bits, m.tiles, m.n_tiles, m.fp6->NK, m.L, m.n_chunk_rows, m.thr,
                           o, sc);
    }
}
}  // namespace

void launch_fp6_probe(const MfmaLaunch &m, unsigned *probe, uint32_t stride, hipStream_t s) {
    const uint64_t *ok_bits = reinterpret_cast<const uint64_t *>(m.wplanes + okbits_offset(m.NP));
    ScreenArgs sc{};
    sc.nonneg = m.nonneg;
    fp6_screen_args(m, sc);
    sc.probe = probe;
    sc.probe_stride = std::max<uint32_t>(stride, 1);
    (void)hipMemsetAsync(probe, 0, 2 * sizeof(unsigned), s);
    launch_fp6_screen(m, ok_bits, OrderArgs{}, sc, sc.probe_stride, s);
}

bool launch_pair_mfma(const MfmaLaunch &m, const OrderArgs &o, const DenseArgs *dense, hipStream_t s,
                      hipEvent_t screen_done) {
    const DenseArgs dn = dense ? *dense : DenseArgs{nullptr, nullptr, nullptr, nullptr};
    const uint64_t *ok_bits = reinterpret_cast<const uint64_t *>(m.wplanes + okbits_offset(m.NP));
    const bool prefilter = !dense && m.prefilter && m.thr > 0.0f;
    ScreenArgs sc{0.0,         0.0f,         0.0f,      0.0f,        0, m.nonneg, m.cand_list, m.cand_count,
                  m.cand_list + 16 * (size_t)m.n_tiles, m.cand_work, m.cand_buckets, m.n_tiles, 0, ScanArgs{}};
    if (!m.frag) {  // site-major kernel (all three planes)
        const dim3 g(m.n_tiles), b(256);
        if (dense)
            hipLaunchKernelGGL((pair_mfma_rows_kernel<kModeDense>), g, b, 0, s, m.codes, m.wplanes, ok_bits, m.tiles,
                               m.L, m.NP, m.n_chunk_rows, m.thr, m.shift, o, dn, sc);
        else if (prefilter)
            hipLaunchKernelGGL((pair_mfma_rows_kernel<kModePrefilter>), g, b, 0, s, m.codes, m.wplanes, ok_bits,
                               m.tiles, m.L, m.NP, m.n_chunk_rows, m.thr, m.shift, o, dn, sc);
        else
            hipLaunchKernelGGL((pair_mfma_rows_kernel<kModeAll>), g, b, 0, s, m.codes, m.wplanes, ok_bits, m.tiles,
                               m.L, m.NP, m.n_chunk_rows, m.thr, m.shift, o, dn, sc);
        return false;
    }
    // the nonzero digit planes in ascending order, 2 bits each; no plane is
    // all zero only if some weight is nonzero, which the caller guarantees
    unsigned mask = m.plane_mask & 15;
    if (!mask) mask = 15;
    uint32_t idx = 0, n = 0, top = 0;
    for (uint32_t p = 0; p < kMaxPlanes; ++p)
        if (mask >> p & 1) idx |= p << (2 * n++), top = p;
    // three active planes other than 0-2 (a 4-plane shift with one all-zero
    // plane) run as four: NPL 3 always means planes 0, 1, 2
    if (n == 3 && idx != kPlanes012) n = 4;
    if (n == 4) idx = 0 | (1 << 2) | (2 << 4) | (3 << 6);
    if (dense) {
        launch_lds_planes<kModeDense>(n, m, ok_bits, m.tiles, m.n_tiles, nullptr, m.n_tiles, idx, o, dn, sc, s);
        return false;
    }
    if (!prefilter) {
        launch_lds_planes<kModeAll>(n, m, ok_bits, m.tiles, m.n_tiles, nullptr, m.n_tiles, idx, o, dn, sc, s);
        return false;
    }
    if (m.ref_rows) {
        // candidate pairs, then each summed alone in lib.rs's order;
        // screen_done separates the two launches, and the second runs the
        // chunk scan.  The bound's residual is the reference's rounding
        // (r_extra_q), which at these thresholds dwarfs what the lowest digit
        // plane adds (2^-16 of the weights against ~1e-4 at N = 2000): with
        // three or more active planes the top two suffice (2/3 of the MFMA
        // work), the planes below bounded by resid as in the two-plane screen;
        // sums in fixed-point units either way
        if (n >= 3) {
            const uint32_t lo = top - 1;
            sc.R = (double)m.resid[lo - 1] + m.r_extra_q;
            launch_lds<kModeRefPairs, 2>(m, ok_bits, m.tiles, m.n_tiles, nullptr, m.n_tiles, lo | (top << 2), o, dn,
                                          sc, s);
        } else {
            sc.R = m.r_extra_q;
            launch_lds_planes<kModeRefPairs>(n, m, ok_bits, m.tiles, m.n_tiles, nullptr, m.n_tiles, idx, o, dn, sc,
                                             s);
        }
        if (screen_done) (void)hipEventRecord(screen_done, s);
        RefRowsLaunch rr = *m.ref_rows;
        rr.slices = m.cand_list;
        rr.slice_count = m.cand_count;
        rr.work = m.cand_work;
        rr.scan = m.scan;
        launch_ref_rows(rr, o, s);
        return true;
    }
    if (!m.screen) {
        launch_lds_planes<kModePrefilter>(n, m, ok_bits, m.tiles, m.n_tiles, nullptr, m.n_tiles, idx, o, dn, sc, s);
        return false;
    }
    sc.scan = m.scan;  // from here on a screen runs (and a candidate launch after it)
    // lib.rs's order on the f32 kernel: candidates as 16-row-block items
    // (buckets 0-3 of capacity 4 n_tiles: the 16 n_tiles list entries)
    if (m.ref_valu && !m.ref_valu->safe) {
        sc.rb_items = 1;
        sc.cand_cap = 4 * m.n_tiles;
    }
    // Screen: the top plane alone over every tile, the residual of the lower
    // planes bounded by R (in top-digit units: exact, a power-of-two scaling
    // of an integer below 2^53); candidate tiles then get every plane.  With
    // one nonzero plane (equal weights, e.g. --unweighted) the screen's sums
    // are exact (R = 0): it only moves the per-pair work to the cheap f32
    // bound, and the candidate launch (two-plane instantiation) adds an
    // all-zero plane.
    if (m.screen2 && n >= 3) {
        // Two-plane screen (low thresholds, where the top plane's residual
        // leaves most tiles undecided): planes lo = top - 1 and top, sums in
        // units of plane lo, the planes below lo bounded by resid[lo - 1]
        // (top >= 2 with three or more active planes, so lo >= 1).  Per pair
        // r2_bound_skip in f64; candidates then get every plane as below.
        const uint32_t lo = top - 1;
        sc.R = ldexp((double)m.resid[lo - 1] + m.r_extra_q, -8 * (int)lo);
        sc.Rf = (float)sc.R;
        if ((double)sc.Rf < sc.R) sc.Rf = nextafterf(sc.Rf, INFINITY);
        sc.f32 = 0;
        launch_lds<kModeScreen, 2>(m, ok_bits, m.tiles, m.n_tiles, nullptr, m.n_tiles, lo | (top << 2), o, dn, sc, s);
        if (screen_done) (void)hipEventRecord(screen_done, s);
        launch_candidates(m, n, idx, ok_bits, o, dn, sc, s);
        return true;
    }
    if (m.fp6) {
        fp6_screen_args(m, sc);
        sc.bail = m.fp6_bail;
        launch_fp6_screen(m, ok_bits, o, sc, 1, s);
        if (screen_done) (void)hipEventRecord(screen_done, s);
        launch_candidates(m, n, idx, ok_bits, o, dn, sc, s);
        return true;
    }
    sc.R = ldexp((top > 0 ? (double)m.resid[top - 1] : 0.0) + m.r_extra_q, -8 * (int)top);
    if (n == 1) idx = top | ((top == 0 ? 1u : 0u) << 2);
    sc.Rf = (float)sc.R;
    if ((double)sc.Rf < sc.R) sc.Rf = nextafterf(sc.Rf, INFINITY);
    // 2: doubled sums (NP <= 16384), 1: halved sums with f64 fallback, 0: f64
    sc.f32 = m.nonneg ? (m.NP <= kScrF32MaxNP ? 2 : m.NP <= kScreenF32MaxNP ? 1 : 0) : 0;
    if (sc.f32 == 2 && m.i8img && m.f6_pairs && m.i8img->digit_plane == top) {
        // tile pairs, wide waves, pre-multiplied operands: the xy2 epilogue on
        // exact marginals needs R2 = 2 R on the integer grid (rounded up: a
        // larger residual bound is still one)
        sc.Rf = (float)(std::ceil(2.0 * sc.R) / 2.0);
        screen_consts((float)(2 * m.dsum[top]), 2.0f * sc.Rf, sc.E, sc.mloc);
        hipLaunchKernelGGL(pair_i8_screen2w_kernel, dim3(m.f6_n_pairs), dim3(256), 0, s, m.i8img->a8, m.i8img->b8,
                           ok_bits, m.f6_pairs, m.f6_n_pairs, (uint32_t)(m.NP / 64), m.L, m.n_chunk_rows, m.thr, o, sc);
        if (screen_done) (void)hipEventRecord(screen_done, s);
        launch_candidates(m, n, idx, ok_bits, o, dn, sc, s);
        return true;
    }
    // every doubled one-plane T <= 2 sum_k |d_top,k| <= 256 NP <= 2^22 (exact in f32)
    if (sc.f32 == 2) screen_consts((float)(2 * m.dsum[top]), 2.0f * sc.Rf, sc.E, sc.mloc);
    launch_lds<kModeScreen, 1>(m, ok_bits, m.tiles, m.n_tiles, nullptr, m.n_tiles, top, o, dn, sc, s);
    if (screen_done) (void)hipEventRecord(screen_done, s);
    launch_candidates(m, n, idx, ok_bits, o, dn, sc, s);
    return true;
}

}  // namespace wld
