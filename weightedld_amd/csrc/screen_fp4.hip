// The fp4 screen: the one-plane screen's job (bound every pair's r2 from
// approximate sums, so that only candidate tiles are computed exactly) on the
// block-scaled fp4 matrix cores, which multiply twice the i8 rate
// (v_mfma_scale_f32_32x32x64_f8f6f4: 32x32x64 in the cycles of a 32x32x32
// i8 MFMA; MI355X_MICROARCH.md, Matrix cores).
//
//   * Weights: q_k = nearest e2m1 value of w_k s (s = g / max w, g in
//     {6, 4, 3, 2}, the one with the smallest residual), chosen on the host
//     with R = sum_k |w_k s - q_k| (rounded up).  Sums of q over any subset of
//     sequences are then within R (L1 over the 2x2 cells) of the exact sums
//     scaled by s: r2_screen_violation's premise (pair_common.hpp).
//   * Operands (frag4_kernel, once per load): A = q where the a site's symbol
//     is in (major or minor) and A' = q where it is the major, both as fp4
//     nibbles (the weight is folded in: no VALU on the A side); B = 1.0 for a
//     minor, 2.0 for a major (0x2 / 0x4 nibbles), so B & 0x22222222 is the
//     minor indicator (the X = S(minor) + 2 S(major), Y = S(minor) form of the
//     i8 kernels).  Products of fp4 values are multiples of 1/2 and every sum
//     stays below 2^22: the f32 accumulators are exact (tools/probes/
//     fp4_probe.hip checks operand pairing and exactness on the device).
//   * Tiles: 64 a sites x 128 b sites per workgroup (the host's wide list:
//     (ta, tb) and, with kWideSecond, (ta, tb + 1)); wave w computes a rows
//     32 (w & 1).. against b columns 64 (w >> 1).. (8 MFMAs and 8 v_and per 64
//     sequences; 128 accumulator registers).  Per 64-sequence stage the eight
//     1 KB operand blocks (A, A' of the two 32-site a blocks, B of the four b
//     blocks) arrive by LDS-DMA, two per wave, double-buffered in groups.
//   * Per pair: r2_screen_violation on the doubled sums (2T = X + Y, ...,
//     exact) with 2R; a 64x64 half with any pair it cannot reject is appended
//     to the candidate list, the others write their zero segment counts.
#include <algorithm>
#include <cmath>
#include <vector>

#include "pair_common.hpp"

namespace wld {

namespace {
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

constexpr int kS4KG = 4;                       // 64-sequence stages per LDS group
constexpr int kS4Stage = 8192;                 // A0 A1 A'0 A'1 B0 B1 B2 B3, 1 KB each
constexpr int kS4Group = kS4KG * kS4Stage;
constexpr unsigned kMinorBits = 0x22222222u;   // the 1.0 (minor) nibbles of a B operand

__device__ __forceinline__ v16f mfma_fp4(v4i a, v4i b, v16f c) {
    const v8i a8 = {a[0], a[1], a[2], a[3], 0, 0, 0, 0}, b8 = {b[0], b[1], b[2], b[3], 0, 0, 0, 0};
    // formats 4/4 = e2m1; scales 0x7F = 2^0 (e8m0)
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, c, 4, 4, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
}

// frag4: three copies of (LP/32) x (NP/64) blocks of 1 KB — A, A', B — where
// block (g, kb) lane l holds the 32 nibbles of site 32g + (l & 31), sequences
// 64 kb + 32 (l >> 5) + e at nibble e (byte e / 2, low nibble first): the
// 32x32x64 fp4 MFMA operand layout (A[row l&31][k = 32 (l>>5) + e]).
__global__ __launch_bounds__(256) void frag4_kernel(const uint8_t *__restrict__ codes, const uint8_t *__restrict__ w4,
                                                     uint32_t LP, uint32_t NP, uint8_t *__restrict__ frag4) {
    const uint32_t NKB = NP / 64;
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;  // one 16-byte lane record
    if (idx >= (size_t)LP * NKB * 2) return;
    const uint32_t l = idx & 63;
    const size_t t = idx >> 6;
    const uint32_t kb = t % NKB;
    const size_t g = t / NKB;
    const uint32_t k0 = kb * 64 + (l >> 5) * 32;
    const uint8_t *c = codes + (g * 32 + (l & 31)) * NP + k0;
    const uint4 c0 = *reinterpret_cast<const uint4 *>(c), c1 = *reinterpret_cast<const uint4 *>(c + 16);
    const uint4 wv = *reinterpret_cast<const uint4 *>(w4 + k0 / 2);
    const uint32_t cw[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    const uint32_t ww[4] = {wv.x, wv.y, wv.z, wv.w};
    uint32_t a[4] = {0, 0, 0, 0}, am[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
#pragma unroll
    for (int e = 0; e < 32; ++e) {
        const uint32_t code = (cw[e / 4] >> (8 * (e % 4))) & 0xFF;
        const uint32_t q = (ww[e / 8] >> (4 * (e % 8))) & 0xF;
        const uint32_t sh = 4 * (e % 8);
        if (code & kCodeIn) {
            a[e / 8] |= q << sh;
            if (code & kCodeMaj) am[e / 8] |= q << sh;
            b[e / 8] |= ((code & kCodeMaj) ? 0x4u : 0x2u) << sh;
        }
    }
    const size_t copy = (size_t)LP * NP / 2;
    uint8_t *o = frag4 + idx * 16;
    *reinterpret_cast<uint4 *>(o) = make_uint4(a[0], a[1], a[2], a[3]);
    *reinterpret_cast<uint4 *>(o + copy) = make_uint4(am[0], am[1], am[2], am[3]);
    *reinterpret_cast<uint4 *>(o + 2 * copy) = make_uint4(b[0], b[1], b[2], b[3]);
}

__global__ __launch_bounds__(256, 2) void screen_fp4_kernel(const uint8_t *__restrict__ frag4,
                                                            const uint64_t *__restrict__ ok_bits,
                                                            const uint32_t *__restrict__ wtiles, uint32_t LP,
                                                            uint32_t NP, float thr_c, float R2, OrderArgs o,
                                                            uint32_t *__restrict__ cand_list,
                                                            unsigned *__restrict__ cand_count) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[2 * kS4Group];
    __shared__ uint32_t sCand[2];
    const uint32_t e = wtiles[blockIdx.x];
    if (e == kNoTile) return;  // padding of an XCD-ordered list (whole workgroup)
    const bool two = (e & kWideSecond) != 0;
    const uint32_t ta = (e >> 16) & 0x7FFFu, tb = e & 0xFFFFu;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t ah = wave & 1, bh = wave >> 1;
    const uint32_t NKB = NP / 64;
    const uint32_t n_groups = (NKB + kS4KG - 1) / kS4KG;
    if (tid < 2) sCand[tid] = 0;  // ordered before the epilogue by the loop's barriers

    // wave w copies operand block w (A of a block 2ta + w for w < 2, A' of
    // 2ta + w - 2 otherwise) and block 4 + w (B of b block 2tb + w, or of the
    // second half's 2tb2 + w - 2) of every stage; a partial last group reads
    // past NKB into the allocation's padding, into stages it never reads
    const size_t blk = (size_t)NKB * 1024, copy = (size_t)LP * NP / 2;
    const uint32_t tb2 = two ? tb + 1 : tb;
    const uint8_t *pa = frag4 + (wave >= 2 ? copy : 0) + (2 * ta + (wave & 1)) * blk;
    const uint8_t *pb = frag4 + 2 * copy + (wave < 2 ? 2 * tb + wave : 2 * tb2 + wave - 2) * blk;
    const uint32_t smem_lds = lds_addr(smem);
    auto issue = [&](uint32_t grp, uint32_t buf) {
        const uint32_t gb = smem_lds + buf * kS4Group;
        const uint32_t voff = grp * (kS4KG * 1024) + lane * 16;
#pragma unroll
        for (int st = 0; st < kS4KG; ++st) {
            glds16_s(pa + st * 1024, voff, gb + st * kS4Stage + wave * 1024);
            glds16_s(pb + st * 1024, voff, gb + st * kS4Stage + (4 + wave) * 1024);
        }
    };

    const uint32_t offA = ah * 1024 + lane * 16, offAm = (2 + ah) * 1024 + lane * 16;
    const uint32_t offB = (4 + 2 * bh) * 1024 + lane * 16;  // + n * 1024
    v16f acc[2][2][2];  // [b block n][A or A'][X, Y]
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y) acc[n][x][y] = v16f{};
    issue(0, 0);
    uint32_t buf = 0;
    for (uint32_t grp = 0; grp < n_groups; ++grp) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's copies of this group landed
        __builtin_amdgcn_s_barrier();                     // ... and every other wave's; the other buffer is free
        asm volatile("" ::: "memory");
        if (grp + 1 < n_groups) issue(grp + 1, buf ^ 1);
        const uint8_t *gb = smem + buf * kS4Group;
        const uint32_t n_st = min((uint32_t)kS4KG, NKB - grp * kS4KG);
        for (uint32_t st = 0; st < n_st; ++st) {
            const uint8_t *s_ = gb + st * kS4Stage;
            const v4i a = *reinterpret_cast<const v4i *>(s_ + offA);
            const v4i am = *reinterpret_cast<const v4i *>(s_ + offAm);
#pragma unroll
            for (int n = 0; n < 2; ++n) {
                const v4i b = *reinterpret_cast<const v4i *>(s_ + offB + n * 1024);
                v4i bm;
#pragma unroll
                for (int k = 0; k < 4; ++k) bm[k] = b[k] & (int)kMinorBits;
                acc[n][0][0] = mfma_fp4(a, b, acc[n][0][0]);
                acc[n][0][1] = mfma_fp4(a, bm, acc[n][0][1]);
                acc[n][1][0] = mfma_fp4(am, b, acc[n][1][0]);
                acc[n][1][1] = mfma_fp4(am, bm, acc[n][1][1]);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads of this buffer done before the next barrier
        buf ^= 1;
    }

    // ---- per-pair bound.  Register i of block n: a = 32 ah + (i & 3) + 8 (i >> 2)
    // + 4 (lane >> 5), b = 32 n + (lane & 31) within half bh (32x32 C/D layout).
    const uint32_t tbh = tb + bh;
    const bool here = bh == 0 || two;  // this wave's 64x64 half exists
    float worst = -1.0f;
    if (here) {
        const uint64_t okA = ok_bits[ta], okB = ok_bits[tbh];
        auto viol = [&](int n, int i) {
            const float X0 = acc[n][0][0][i], Y0 = acc[n][0][1][i], X1 = acc[n][1][0][i], Y1 = acc[n][1][1][i];
            // doubled sums 2T, 2SA, 2SB, 2SAB (exact in f32)
            return r2_screen_violation(X0 + Y0, X1 + Y1, X0 - Y0, X1 - Y1, R2, thr_c);
        };
        if (okA == ~0ull && okB == ~0ull && ta != tbh) {  // every pair valid (the common case)
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
                for (int i = 0; i < 16; ++i) worst = fmaxf(worst, viol(n, i));
        } else {
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const uint32_t al = 32 * ah + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5), bl = 32 * n + (lane & 31);
                    const bool valid = ((okA >> al) & 1) && ((okB >> bl) & 1) && (ta != tbh || al < bl);
                    if (valid) worst = fmaxf(worst, viol(n, i));
                }
        }
    }
    const bool cand = !(worst <= 0.0f);  // some valid pair the bound cannot reject
    if (__builtin_amdgcn_ballot_w64(cand) != 0 && lane == 0) sCand[bh] = 1;
    __syncthreads();
    const uint32_t half = tid >> 6;  // threads 0-63: tile (ta, tb); 64-127: (ta, tb + 1)
    if (half < 2 && (half == 0 || two)) {
        const uint32_t t = tb + half;
        if (sCand[half]) {
            if (lane == 0) cand_list[atomicAdd(cand_count, 1u)] = (ta << 16) | t;
        } else {
            o.seg_cnt[(size_t)(ta * kTile + lane) * o.T + t] = 0;
        }
    }
}
}  // namespace

size_t screen_fp4_frag_bytes(size_t LP, size_t NP) { return LP * NP / 2 * 3 + kS4KG * 1024; }

void launch_frag4(const uint8_t *codes, const uint8_t *w4, size_t LP, size_t NP, uint8_t *frag4, hipStream_t s) {
    const size_t recs = LP * (NP / 64) * 2;
    hipLaunchKernelGGL(frag4_kernel, dim3((unsigned)((recs + 255) / 256)), dim3(256), 0, s, codes, w4, (uint32_t)LP,
                       (uint32_t)NP, frag4);
}

void launch_screen_fp4(const uint8_t *frag4, const uint64_t *ok_bits, const uint32_t *wtiles, uint32_t n_wtiles,
                       size_t LP, size_t NP, float thr, float R, const OrderArgs &o, uint32_t *cand_list,
                       unsigned *cand_count, hipStream_t s) {
    const float thr_c = thr * (1.0f - 0x1p-7f);
    hipLaunchKernelGGL(screen_fp4_kernel, dim3(n_wtiles), dim3(256), 0, s, frag4, ok_bits, wtiles, (uint32_t)LP,
                       (uint32_t)NP, thr_c, 2.0f * R, o, cand_list, cand_count);
}

// e2m1 magnitudes by code 0..7
static const double kFp4[8] = {0.0, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0};

int fp4_weights(const float *w, size_t N, size_t NP, std::vector<uint8_t> &packed, float *R_out) {
    double maxw = 0.0;
    for (size_t k = 0; k < N; ++k) {
        if (!(w[k] >= 0.0f) || !std::isfinite(w[k])) return -1;  // nonnegative finite weights only
        maxw = std::max(maxw, (double)w[k]);
    }
    if (!(maxw > 0.0)) return -1;
    double best = -1.0, best_R = 0.0, best_s = 0.0;
    for (double g : {6.0, 4.0, 3.0, 2.0}) {
        const double s = g / maxw;
        double R = 0.0, T = 0.0;
        for (size_t k = 0; k < N; ++k) {
            const double x = (double)w[k] * s;
            double q = 0.0, d = 1e300;
            for (double v : kFp4)
                if (std::fabs(x - v) < d) d = std::fabs(x - v), q = v;
            R += d;
            T += x;
        }
        const double rel = R / T;
        if (best < 0.0 || rel < best) best = rel, best_R = R, best_s = s;
    }
    packed.assign(NP / 2, 0);
    for (size_t k = 0; k < N; ++k) {
        const double x = (double)w[k] * best_s;
        int code = 0;
        double d = 1e300;
        for (int c = 0; c < 8; ++c)
            if (std::fabs(x - kFp4[c]) < d) d = std::fabs(x - kFp4[c]), code = c;
        packed[k / 2] |= (uint8_t)(code << (4 * (k % 2)));
    }
    // R in units of the scaled weights, with room for the double rounding of
    // w s and of the sum (any R above the true residual keeps the bound sound)
    const double R = best_R * (1.0 + 1e-9) + 1e-9 * (double)N;
    float Rf = (float)R;
    if ((double)Rf < R) Rf = std::nextafter(Rf, INFINITY);
    *R_out = Rf;
    return 0;
}

}  // namespace wld
