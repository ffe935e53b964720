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
//   * A operand (a sites): indicator byte mask & digit byte (in & d_p, maj & d_p);
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
// shard's chunk rows); wave w owns the 32x32 sub-tile (w>>1, w&1).  Operands
// stream through LDS in groups of kGroup 32-sequence stages, double-buffered
// and filled with global_load_lds (async, no VGPRs): per stage each wave copies
// one 1 KB code-fragment block (A0, A1, B0, B1 of the fragment-major layout),
// and per group wave 0 copies the group's 1 KB of weight digits (128 B per
// stage).  Every DMA is a full-wave 1 KB copy, and a group is consumed only
// after s_waitcnt vmcnt(0) + a barrier — correctness never depends on the
// completion order of outstanding loads.  The next group's copies are issued
// right after that barrier, one group (8 stages of MFMA work) ahead of use.
// Passing rows are compacted per 64x64 tile in LDS (order.hip assembles the
// reference order).
#include "pair_common.hpp"

namespace wld {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void;

bool mfma_supported() { return true; }

#ifdef WLD_EXP_STAMPS
// diagnostic build only: per-phase cycle sums over all waves (s_memtime)
__device__ unsigned long long g_stamp[8];
__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define WLD_STAMP(v) const unsigned long long v = stamp()
#else
#define WLD_STAMP(v)
#endif

namespace {
constexpr int kGroup = 8;                           // 32-sequence stages per LDS group
constexpr int kStageCodes = 4096;                   // A0 A1 B0 B1, 1 KB each
constexpr int kDigStage = 128;                      // digit bytes per stage: [plane][half][16] + 32 pad
constexpr int kGroupBytes = kGroup * (kStageCodes + kDigStage);  // 33 KB; two groups in LDS
}  // namespace

// Weight digits of q = rint(w * 2^shift) in two layouts:
//   planes[p*NP + k]                      (plane-major, site-major kernel path)
//   digf[kb*128 + (2p + h)*16 + j]        (per 32-sequence stage, LDS path;
//                                          k = 32kb + 16h + j; bytes 96..127 pad)
__global__ __launch_bounds__(256) void mfma_prep_kernel(const float *__restrict__ w_pad, uint32_t NP, int shift,
                                                         int8_t *__restrict__ planes, int8_t *__restrict__ digf) {
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= NP) return;
    long long q = llrint(ldexp((double)w_pad[k], shift));
    const uint32_t kb = k >> 5, h = (k >> 4) & 1, j = k & 15;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        const long long r = ((q + 128) & 255) - 128;  // balanced digit in [-128, 127]
        q = (q - r) / 256;
        planes[p * NP + k] = (int8_t)r;
        digf[kb * kDigStage + (2 * p + h) * 16 + j] = (int8_t)r;
    }
}

// codes_frag: the (site, sequence) codes in "fragment-major" order, so a
// wave's A or B operand for 32 sites x 32 sequences is one contiguous 1 KB
// block (lane l = 32h + r gets site r, sequences 16h..16h+15 — the MFMA
// operand layout):
//   frag[((g * NKB + kb) * 64 + l) * 16 + j] = sel(codes[(32g + (l&31)) * NP + 32kb + 16(l>>5) + j])
// Each byte is stored as a v_perm_b32 selector for its byte position j&3:
//   12 (not major/minor -> constant 0x00), j&3 (minor), 4 + (j&3) (major),
// so one v_perm_b32 per dword turns codes + weight digits straight into MFMA
// operands (perm_operands below) with no mask arithmetic.
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
    uint32_t in[4] = {v.x, v.y, v.z, v.w}, out[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        uint32_t o = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t c = (in[e] >> (8 * j)) & 0xFF;
            const uint32_t sel = (c & kCodeIn) ? ((c & kCodeMaj) ? 4u + j : (uint32_t)j) : 12u;
            o |= sel << (8 * j);
        }
        out[e] = o;
    }
    *reinterpret_cast<uint4 *>(frag + idx * 16) = make_uint4(out[0], out[1], out[2], out[3]);
}

__device__ __forceinline__ v16i mfma_i8(v4i a, v4i b, v16i c) {
    return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
}

// Byte-wise masks from code bytes c in {0 (out), 1 (minor), 3 (major)}:
// v_perm_b32 with zero sources returns, per selector byte, 0xFF for >= 13 and
// 0x00 for 8..12 — a byte compare without a multiply.
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

// 12 MFMAs of one 32-sequence block from selector-coded fragments (frag_kernel):
// v_perm_b32(S0, S1, sel) takes byte sel of {S0:S1} (0-3 from S1, 4-7 from S0,
// 12 -> 0x00), so with S0 = S1 = digits a selector yields the digit for minor
// and major, with S1 = 0 only for major; with 0x01 bytes the 0/1 indicators.
__device__ __forceinline__ void mfma_block_sel(v16i (&acc)[2][3][2], v4i ca, v4i cb, v4i d0, v4i d1, v4i d2) {
    constexpr unsigned kOnes = 0x01010101u;
    v4i b_in, b_maj;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        b_in[e] = (int)__builtin_amdgcn_perm(kOnes, kOnes, (unsigned)cb[e]);
        b_maj[e] = (int)__builtin_amdgcn_perm(kOnes, 0u, (unsigned)cb[e]);
    }
    const v4i dp[3] = {d0, d1, d2};
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        v4i ai, am;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            ai[e] = (int)__builtin_amdgcn_perm((unsigned)dp[p][e], (unsigned)dp[p][e], (unsigned)ca[e]);
            am[e] = (int)__builtin_amdgcn_perm((unsigned)dp[p][e], 0u, (unsigned)ca[e]);
        }
        acc[0][p][0] = mfma_i8(ai, b_in, acc[0][p][0]);
        acc[0][p][1] = mfma_i8(ai, b_maj, acc[0][p][1]);
        acc[1][p][0] = mfma_i8(am, b_in, acc[1][p][0]);
        acc[1][p][1] = mfma_i8(am, b_maj, acc[1][p][1]);
    }
}

// 12 MFMAs of one 32-sequence block for this wave's 32x32 sub-tile (site-major codes)
__device__ __forceinline__ void mfma_block(v16i (&acc)[2][3][2], v4i ca, v4i cb, v4i d0, v4i d1, v4i d2) {
#ifdef WLD_EXP_NOVALU
    {  // diagnostic: the 12 MFMAs without the operand VALU
        const v4i dq[3] = {d0, d1, d2};
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y)
                    acc[x][p][y] = mfma_i8(x ? ca : dq[p], y ? cb : dq[(p + 1) % 3], acc[x][p][y]);
        return;
    }
#endif
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

// DENSE: write every pair's stats (tests).  RING: fragment-major codes through
// the double-buffered LDS groups (else site-major codes read straight into registers).
// PREFILTER (threshold > 0): skip the f32 epilogue for pairs whose exact r2,
// evaluated in f64 from the exact integer sums, lies clearly below the threshold.
#ifdef WLD_EXP_LB1
#define WLD_MFMA_WAVES_PER_SIMD 1
#else
#define WLD_MFMA_WAVES_PER_SIMD 2
#endif
template <bool DENSE, bool RING, bool PREFILTER>
__global__ __launch_bounds__(256, WLD_MFMA_WAVES_PER_SIMD) void pair_mfma_kernel(const uint8_t *__restrict__ codes,
                                                            const int8_t *__restrict__ planes,
                                                            const uint8_t *__restrict__ site_ok,
                                                            const uint32_t *__restrict__ tiles, uint32_t L,
                                                            uint32_t NP, uint32_t n_chunk_rows, float thr, int shift,
                                                            OrderArgs o, DenseArgs dn) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[2 * kGroupBytes];  // the only LDS object

    WLD_STAMP(t0);
    const uint32_t tile = tiles[blockIdx.x];
    const uint32_t ta = tile >> 16, tb = tile & 0xFFFFu;
    const uint32_t a0 = ta * kTile, b0 = tb * kTile;
    const uint32_t tid = threadIdx.x;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const uint32_t wa = wave >> 1, wb = wave & 1;
    const uint32_t r = lane & 31, h = lane >> 5;
    const uint32_t NKB = NP / 32;

    // site filter of the tile's 64 a and 64 b sites as wave-uniform bit masks
    // (loaded once, ahead of the main loop, instead of per pair in the epilogue)
    const uint64_t okA = __ballot(a0 + lane < L && site_ok[a0 + lane]);
    const uint64_t okB = __ballot(b0 + lane < L && site_ok[b0 + lane]);

    v16i acc[2][3][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int y = 0; y < 2; ++y)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[x][p][y][e] = 0;

    if constexpr (RING) {
        // this wave's code block per stage (A0/A1/B0/B1); wave 0 also the digit records
        const uint32_t g_src = wave < 2 ? (a0 >> 5) + wave : (b0 >> 5) + (wave - 2);
        const uint8_t *src = codes + ((size_t)g_src * NKB * 64 + lane) * 16;
        const int8_t *dsrc = planes + 3 * (size_t)NP + lane * 16;  // digf
        const uint32_t n_groups = (NKB + kGroup - 1) / kGroup;
#ifdef WLD_EXP_STAMPS
        unsigned long long t1 = 0;
#endif
        auto issue = [&](uint32_t grp) {
            uint8_t *gb = smem + (grp & 1) * kGroupBytes;
            const uint32_t kb0 = grp * kGroup;
#pragma unroll
            for (int st = 0; st < kGroup; ++st)
                if (kb0 + st < NKB)
                    __builtin_amdgcn_global_load_lds(src + (size_t)(kb0 + st) * 1024,
                                                     (lds_void *)(gb + st * kStageCodes + wave * 1024), 16, 0, 0);
            if (wave == 0)  // digits of 8 stages = 1 KB (allocation padded to whole groups)
                __builtin_amdgcn_global_load_lds(dsrc + (size_t)kb0 * kDigStage,
                                                 (lds_void *)(gb + kGroup * kStageCodes), 16, 0, 0);
        };
        issue(0);
        for (uint32_t grp = 0; grp < n_groups; ++grp) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's copies of group grp landed
            __builtin_amdgcn_s_barrier();                     // ... and every other wave's; group grp-1 is free
            asm volatile("" ::: "memory");
#ifdef WLD_EXP_STAMPS
            if (grp == 0) t1 = stamp();
#endif
#ifdef WLD_EXP_NOLOAD
            if (grp + 1 < n_groups && grp == 0) issue(grp + 1);  // diagnostic: no streaming
#else
            if (grp + 1 < n_groups) issue(grp + 1);
#endif
            const uint8_t *gb = smem + (grp & 1) * kGroupBytes;
            const uint32_t n_st = min((uint32_t)kGroup, NKB - grp * kGroup);
#ifdef WLD_EXP_PIPE
            auto ld = [&](uint32_t st, v4i &ca, v4i &cb, v4i &d0, v4i &d1, v4i &d2) {
                const uint8_t *sc = gb + st * kStageCodes;
                const uint8_t *sd = gb + kGroup * kStageCodes + st * kDigStage + h * 16;
                ca = *reinterpret_cast<const v4i *>(sc + wa * 1024 + lane * 16);
                cb = *reinterpret_cast<const v4i *>(sc + 2048 + wb * 1024 + lane * 16);
                d0 = *reinterpret_cast<const v4i *>(sd);
                d1 = *reinterpret_cast<const v4i *>(sd + 32);
                d2 = *reinterpret_cast<const v4i *>(sd + 64);
            };
            v4i ca, cb, d0, d1, d2;
            ld(0, ca, cb, d0, d1, d2);
            for (uint32_t st = 0; st < n_st; ++st) {
                v4i na = ca, nb = cb, n0 = d0, n1 = d1, n2 = d2;
                if (st + 1 < n_st) ld(st + 1, na, nb, n0, n1, n2);
                mfma_block_sel(acc, ca, cb, d0, d1, d2);
                ca = na; cb = nb; d0 = n0; d1 = n1; d2 = n2;
            }
#else
#ifdef WLD_EXP_PURE
            for (uint32_t st = 0; st < n_st; ++st) {
                v4i ca = {(int)lane, (int)st, (int)grp, 3}, cb = {(int)(lane ^ 5), 1, 2, (int)st};
                asm volatile("" : "+v"(ca), "+v"(cb));
                mfma_block(acc, ca, cb, ca, cb, ca);
            }
            if (false)
#endif
            for (uint32_t st = 0; st < n_st; ++st) {
                const uint8_t *sc = gb + st * kStageCodes;
                const uint8_t *sd = gb + kGroup * kStageCodes + st * kDigStage + h * 16;
                const v4i ca = *reinterpret_cast<const v4i *>(sc + wa * 1024 + lane * 16);
                const v4i cb = *reinterpret_cast<const v4i *>(sc + 2048 + wb * 1024 + lane * 16);
                const v4i d0 = *reinterpret_cast<const v4i *>(sd);
                const v4i d1 = *reinterpret_cast<const v4i *>(sd + 32);
                const v4i d2 = *reinterpret_cast<const v4i *>(sd + 64);
#ifdef WLD_EXP_EARLYD2
                asm volatile("" ::"v"(d2[0]), "v"(d2[1]), "v"(d2[2]), "v"(d2[3]));
#endif
                mfma_block_sel(acc, ca, cb, d0, d1, d2);
#ifdef WLD_EXP_SGB
                __builtin_amdgcn_sched_group_barrier(0x100, 5, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
#pragma unroll
                for (int q = 0; q < 10; ++q) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
                }
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
#endif
            }
#endif
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads of group grp done before the barrier
        }
        __syncthreads();  // LDS reads done before the compaction reuses smem
#ifdef WLD_EXP_STAMPS
        WLD_STAMP(t2);
        if (lane == 0) {
            atomicAdd(&g_stamp[0], t1 - t0);
            atomicAdd(&g_stamp[1], t2 - t1);
            atomicAdd(&g_stamp[5], 1ull);
        }
#endif
    } else {
        const uint8_t *pa = codes + (size_t)(a0 + 32 * wa + r) * NP + 16 * h;
        const uint8_t *pb = codes + (size_t)(b0 + 32 * wb + r) * NP + 16 * h;
        const int8_t *pd = planes + 16 * h;
        for (uint32_t k0 = 0; k0 < NP; k0 += 32) {
            const v4i ca = *reinterpret_cast<const v4i *>(pa + k0);
            const v4i cb = *reinterpret_cast<const v4i *>(pb + k0);
            const v4i d0 = *reinterpret_cast<const v4i *>(pd + k0);
            const v4i d1 = *reinterpret_cast<const v4i *>(pd + NP + k0);
            const v4i d2 = *reinterpret_cast<const v4i *>(pd + 2 * NP + k0);
            mfma_block(acc, ca, cb, d0, d1, d2);
        }
    }

    // ---- epilogue: lane holds b = b0+32wb+r and 16 a rows -------------------
    const double scale = ldexp(1.0, -shift);
    const uint32_t b_local = 32 * wb + r;
    const uint32_t b = b0 + b_local;
    const bool okb = (okB >> b_local) & 1;
    float res[16][3];
    uint32_t pass = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t a_local = 32 * wa + (i & 3) + 8 * (i >> 2) + 4 * h;
        const uint32_t a = a0 + a_local;
        const bool valid = okb && a < b && ((okA >> a_local) & 1);
        // S = acc_0 + 2^8 acc_1 + 2^16 acc_2: integers below 2^48, exact in f64
        double S[2][2];
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y)
                S[x][y] = fma(65536.0, (double)acc[x][2][y][i],
                              fma(256.0, (double)acc[x][1][y][i], (double)acc[x][0][y][i]));
        if constexpr (!DENSE) {
            if (!valid) continue;
            if constexpr (PREFILTER) {
                // Exact algebra: d = PA*PB - P(AB) and r2 = d^2/(PA Pa PB Pb) become
                // r2 = (SA*SB - SAB*T)^2 / (SA (T-SA) SB (T-SB)) on the exact sums.
                // Evaluated in f64 (|err| ~1e-16 relative); pairs more than
                // 1e-5 + 1e-4|thr| below the threshold cannot pass the f32
                // epilogue, so they skip it.  Everything else (and den <= 0,
                // the NaN/inf cases) takes the full reference epilogue.
                const double T = S[0][0], SA = S[1][0], SB = S[0][1], SAB = S[1][1];
                const double num = SA * SB - SAB * T;
                const double den = SA * (T - SA) * SB * (T - SB);
                const double cut = (double)thr - (1e-5 + 1e-4 * fabs((double)thr));
                if (den > 0.0 && num * num < cut * den) continue;
            }
        }
        float s[2][2];
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y) s[x][y] = (float)(S[x][y] * scale);
        float d, dp, r2;
        ld_epilogue(s[0][0], s[1][0], s[0][1], s[1][1], d, dp, r2);
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
            if (valid && r2 > thr) pass |= 1u << i;  // lib.rs:660 strict '>'
        }
    }
    if constexpr (DENSE) return;
#ifdef WLD_EXP_STAMPS
    WLD_STAMP(t3);
#endif

    // ---- compaction: a 64x64 pass-bit matrix in LDS, rows in b order ----------
    unsigned long long *sBits = reinterpret_cast<unsigned long long *>(smem);  // [64]
    uint32_t *sRowBase = reinterpret_cast<uint32_t *>(smem + kTile * 8);      // [64]
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
#ifdef WLD_EXP_STAMPS
    WLD_STAMP(t4);
    if (lane == 0) {
        atomicAdd(&g_stamp[2], t3 - t0);
        atomicAdd(&g_stamp[3], t4 - t3);
    }
#endif
}

#ifdef WLD_EXP_STAMPS
extern "C" int wld_debug_stamps(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamp), sizeof(g_stamp)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamp), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

size_t mfma_planes_bytes(size_t NP) {
    const size_t n_groups = (NP / 32 + kGroup - 1) / kGroup;
    return 3 * NP + n_groups * kGroup * kDigStage;  // digit records padded to whole groups
}

void launch_mfma_prep(const uint8_t *, const float *w_pad, size_t, size_t NP, int shift, int8_t *planes,
                      hipStream_t s) {
    hipLaunchKernelGGL(mfma_prep_kernel, dim3((unsigned)((NP + 255) / 256)), dim3(256), 0, s, w_pad, (uint32_t)NP,
                       shift, planes, planes + 3 * NP);
}

void launch_frag(const uint8_t *codes, size_t LP, size_t NP, uint8_t *frag, hipStream_t s) {
    const size_t chunks = LP * NP / 16;
    hipLaunchKernelGGL(frag_kernel, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0, s, codes, (uint32_t)LP,
                       (uint32_t)NP, frag);
}

void launch_pair_mfma(const uint8_t *codes, const uint8_t *frag, const int8_t *wplanes, const uint8_t *site_ok,
                      const uint32_t *tiles, uint32_t n_tiles, uint32_t L, uint32_t NP, uint32_t n_chunk_rows,
                      float thr, int shift, bool prefilter, const OrderArgs &o, const DenseArgs *dense,
                      hipStream_t s) {
    const DenseArgs none{nullptr, nullptr, nullptr, nullptr};
    const dim3 g(n_tiles), b(256);
    if (dense) {
        if (frag)
            hipLaunchKernelGGL((pair_mfma_kernel<true, true, false>), g, b, 0, s, frag, wplanes, site_ok, tiles, L, NP,
                               n_chunk_rows, thr, shift, o, *dense);
        else
            hipLaunchKernelGGL((pair_mfma_kernel<true, false, false>), g, b, 0, s, codes, wplanes, site_ok, tiles, L,
                               NP, n_chunk_rows, thr, shift, o, *dense);
    } else if (frag) {
        if (prefilter)
            hipLaunchKernelGGL((pair_mfma_kernel<false, true, true>), g, b, 0, s, frag, wplanes, site_ok, tiles, L, NP,
                               n_chunk_rows, thr, shift, o, none);
        else
            hipLaunchKernelGGL((pair_mfma_kernel<false, true, false>), g, b, 0, s, frag, wplanes, site_ok, tiles, L,
                               NP, n_chunk_rows, thr, shift, o, none);
    } else {
        if (prefilter)
            hipLaunchKernelGGL((pair_mfma_kernel<false, false, true>), g, b, 0, s, codes, wplanes, site_ok, tiles, L,
                               NP, n_chunk_rows, thr, shift, o, none);
        else
            hipLaunchKernelGGL((pair_mfma_kernel<false, false, false>), g, b, 0, s, codes, wplanes, site_ok, tiles, L,
                               NP, n_chunk_rows, thr, shift, o, none);
    }
}

}  // namespace wld
