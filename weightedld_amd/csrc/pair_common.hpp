// Device helpers shared by the pair kernels: the LdStats epilogue and the
// tile compaction that feeds the reference-order gather (order.hip).
#pragma once

#include "kernels.hpp"

namespace wld {

// lib.rs:482-520, operation for operation in f32 (the library is built with
// -ffp-contract=off, divisions are IEEE-rounded, fminf/fmaxf ignore NaN like
// Rust's f32::min/max).  Inputs are the four masked weight sums of
// lib.rs:423-480: total_weight, PA (a major), PB (b major), ld_obs[3] (both).
//
// The eight quotients by total_weight (WLD_EPI_DIVT 1, the default) are the
// IEEE f32 quotients computed as RN_f32(x * r) in f64, r a reciprocal of
// total_weight refined to within a few f64 ulps (one hardware estimate, two
// Newton steps), instead of eight f32 division sequences.  Why that is the
// correctly rounded quotient: a midpoint m between two f32 values (a 25-bit
// odd significand M) can equal x / T only if T is a power of two, and then
// x / T is an f32 value itself, so no quotient of two f32 values is a tie;
// and a quotient that is not a midpoint lies at least 1 / (M U) >= 2^-49 of m
// from it (|x - m T| is at least the unit of m T's last place, x = X 2^a with
// 24-bit X, T = U 2^c), while RN_f64(x * r) is within ~2^-51 of x / T: both
// round to the same f32 value (subnormal results too: their midpoints are
// coarser).  T = 0 or non-finite takes the plain divisions (IEEE's inf / NaN).
#ifndef WLD_EPI_DIVT
#define WLD_EPI_DIVT 1
#endif
// (r0: the estimate to refine; the device's v_rcp_f64, the host check's a
// coarser one, the f32 reciprocal)
__host__ __device__ __forceinline__ double recip_f64(double t, double r0) {
    double r = r0;
    double e = fma(-t, r, 1.0);
    r = fma(r, e, r);
    e = fma(-t, r, 1.0);
    return fma(r, e, r);
}
// The host's estimate: the f32 reciprocal, a subnormal t first scaled into
// the normal range (1.0f / t overflows to inf there)
__host__ __forceinline__ double recip_seed_host(float t) {
    return fabsf(t) < 0x1p-126f ? (double)(1.0f / (t * 0x1p64f)) * 0x1p64 : (double)(1.0f / t);
}
__host__ __device__ __forceinline__ void ld_epilogue(float total_weight, float PA, float PB, float ld3, float &d_out,
                                                     float &dp_out, float &r2_out) {
    float ld_obs0, ld_obs1, ld_obs2, ld_obs3 = ld3;
    float Pa = total_weight - PA;
    float Pb = total_weight - PB;
    ld_obs2 = PA - ld_obs3;
    ld_obs1 = PB - ld_obs3;
    ld_obs0 = Pa - ld_obs1;
    if (WLD_EPI_DIVT && total_weight != 0.0f && fabsf(total_weight) <= 3.4028235e38f) {
#if defined(__HIP_DEVICE_COMPILE__)
        const double r = recip_f64((double)total_weight, __builtin_amdgcn_rcp((double)total_weight));
#else
        const double r = recip_f64((double)total_weight, recip_seed_host(total_weight));
#endif
        PA = (float)((double)PA * r);
        PB = (float)((double)PB * r);
        Pa = (float)((double)Pa * r);
        Pb = (float)((double)Pb * r);
        ld_obs0 = (float)((double)ld_obs0 * r);
        ld_obs1 = (float)((double)ld_obs1 * r);
        ld_obs2 = (float)((double)ld_obs2 * r);
        ld_obs3 = (float)((double)ld_obs3 * r);
    } else {
        PA = PA / total_weight;
        PB = PB / total_weight;
        Pa = Pa / total_weight;
        Pb = Pb / total_weight;
        ld_obs0 = ld_obs0 / total_weight;
        ld_obs1 = ld_obs1 / total_weight;
        ld_obs2 = ld_obs2 / total_weight;
        ld_obs3 = ld_obs3 / total_weight;
    }
    const float PAB = PA * PB;
    const float PAb = PA * Pb;
    const float PaB = Pa * PB;
    const float Pab = Pa * Pb;
    const float d = ((PAB - ld_obs3) + (Pab - ld_obs0) + (ld_obs2 - PAb) + (ld_obs1 - PaB)) / 4.0f;
    float den;
    if (d < 0.0f) {
        den = fmaxf(-ld_obs0, -ld_obs3);
        if (den == 0.0f) den = fminf(-ld_obs0, -ld_obs3);
    } else {
        den = fminf(ld_obs1, ld_obs2);
        if (den == 0.0f) den = fmaxf(ld_obs1, ld_obs2);
    }
    d_out = d;
    dp_out = d / den;
    r2_out = d * d / (PA * Pa * PB * Pb);
}

// Rigorous skip test for the r2 > thr filter (thr > 0).  T, A, B, AB are
// approximations of a pair's exact masked sums T, SA, SB, SAB (any common
// unit) whose 2x2 cells n11 = AB, n10 = A-AB, n01 = B-AB, n00 = T-A-B+AB are
// each within e_c of the exact cells, sum_c |e_c| <= R (R = 0: the sums are
// exact).  Returns true only if ld_epilogue, run on the correctly rounded f32
// values of the EXACT sums, cannot give r2 > thr — so skipping the pair never
// changes the output.  Derivation ("Prefilter and screen"):
//   * the f32 epilogue's d is within e_d = 16.25u (u = 2^-24) of the exact
//     D = (SA SB - SAB T) / T^2 (all normalised quantities in [0, 1]), and its
//     denominator PA Pa PB Pb is >= P (1 - 5u sum_i 1/f_i - 3u), f_i the four
//     normalised marginals, so r2_f32 <= (|D| + e_d)^2 (1+u)^2 / (P (1 - rel));
//   * with uncertain sums, |num - num^| <= R max_c |n^_c| + R^2/4, each
//     marginal is within R, T within R.
// Evaluated division-free in f64 with e_d = 24u, rel = 28u T/m + 8u, and a
// 1e-12 relative allowance for the f64 evaluation itself.  Exact cells must be
// >= 0 (normalised quantities in [0, 1]): guaranteed for nonnegative weights,
// else checked as n^_c >= R.
// (__host__ as well: tests/cpp/bound_check.cpp runs the same code on the CPU.)
__host__ __device__ __forceinline__ bool r2_bound_skip(double T, double A, double B, double AB, double R, float thr,
                                                       bool nonneg) {
    constexpr double u = 0x1p-24;
    const double n10 = A - AB, n01 = B - AB, n00 = (T - A) - n01;
    if (!nonneg && fmin(fmin(AB, n10), fmin(n01, n00)) < R) return false;
    const double cmax = fmax(fmax(fabs(AB), fabs(n10)), fmax(fabs(n01), fabs(n00)));
    const double m1 = A - R, m2 = (T - A) - R, m3 = B - R, m4 = (T - B) - R;
    const double mlo = fmin(fmin(m1, m2), fmin(m3, m4));
    if (!(mlo > 0.0)) return false;
    const double Tub = T + R;
    const double nub = fabs(A * B - AB * T) + R * cmax + 0.25 * R * R + (24.0 * u + 0x1p-40) * Tub * Tub;
    const double lhs = nub * nub * ((1.0 + 4.0 * u) * (1.0 + 1e-12)) * mlo;
    const double rhs = (double)thr * ((m1 * m2) * (m3 * m4)) * (mlo * (1.0 - 8.0 * u) - 28.0 * u * Tub);
    return lhs <= rhs;
}

// The screen's per-pair test in f32 (about a third of r2_bound_skip's f64
// cost; the one-plane screen kernel is VALU-issue bound).
// Sound under: nonnegative weights; T, A, B, AB integers of magnitude
// <= 2^22 (exact in f32, and so are T - A, T - B); R >= the L1 cell residual
// (rounded up to f32).  It implies r2_bound_skip's inequality:
//   * every approximate sum and cell is <= Tb = T + 2R (exact cells >= 0 sum
//     to at most T + R, each within R), so R cmax <= R Tb, Tub <= Tb;
//   * |fl(fl(A B) - fl(AB T)) - |A B - AB T|| <= 4.02u Tb^2, so
//     E = R Tb + R^2 + 2^-19 Tb^2 (2^-19 = 32u >= 24u + 2^-40 + 4.02u, the
//     slack covering E's own rounding) gives nub <= fl(num + E)(1 + 2u);
//   * m_i = fl(x_i - R) <= (x_i - R)(1 + u), so the f32 product of the four
//     marginals is <= their exact product times (1 + u)^7;
//   * mlo >= 2^-12 Tb bounds r2_bound_skip's 28u Tub / mlo term by 6.84e-3,
//     and c = 1 - 2^-7 covers it with every f32 rounding above (16u).
// No skip (the tile becomes a candidate) whenever it cannot decide.  Finite
// inputs only (integer sums).  tests/test_r2_bound.py checks it on the host.
// Returned as a violation margin: the pair is skipped iff it is <= 0 (both
// terms are differences of f32 values, whose rounded sign is exact).
// thr_c = thr * (1 - 2^-7) in f32.
// The derivation holds for Tb any f32 upper bound of T + 2R (it only bounds
// sums, cells and T + R from above), so a launch may fix Tb from a bound Tg on
// every T it screens (the screen: Tg = 2 sum_k |top digit_k|, doubled sums)
// and precompute E(Tb) and 2^-12 Tb once (screen_consts); per pair that leaves
// r2_screen_terms, whose two terms must both be <= 0 for a skip.
__host__ __device__ __forceinline__ void screen_consts(float Tg, float R, float &E, float &mloc) {
    const float Tb = (Tg + 2.0f * R) * (1.0f + 0x1p-20f);
    E = R * Tb + R * R + 0x1p-19f * (Tb * Tb);
    mloc = 0x1p-12f * Tb;
}
__host__ __device__ __forceinline__ float r2_screen_terms(float T, float A, float B, float AB, float R, float thr_c,
                                                          float E, float mloc, float &t2) {
    const float m1 = A - R, m2 = (T - A) - R, m3 = B - R, m4 = (T - B) - R;
    const float mlo = fminf(fminf(m1, m2), fminf(m3, m4));
    const float nub = fabsf(A * B - AB * T) + E;
    t2 = mloc - mlo;
    return nub * nub - thr_c * ((m1 * m2) * (m3 * m4));
}
// The same terms straight from the i8 kernel's accumulators in doubled units
// (X0 = S(raw), Y0 = S(minor) of channel_a "in", X1, Y1 of "major"; T = X0 +
// Y0, B = X0 - Y0, A = X1 + Y1, AB = X1 - Y1, all exact): T - B = 2 Y0 and
// A B - AB T = 2 (X0 Y1 - X1 Y0).  The marginals round exactly as in
// r2_screen_terms; the numerator by one FMA (error <= 2u (X0 Y1 + X1 Y0) <= 2u
// T^2, inside the 4.02u Tb^2 the derivation allows) and nub = fl(2 |num'| + E)
// rounds once, as fl(|num| + E) did.
__host__ __device__ __forceinline__ float r2_screen_terms_xy(float X0, float Y0, float X1, float Y1, float R,
                                                             float thr_c, float E, float mloc, float &t2) {
    const float T = X0 + Y0, B = X0 - Y0, A = X1 + Y1;
    const float m1 = A - R, m2 = (T - A) - R, m3 = B - R, m4 = fmaf(2.0f, Y0, -R);
    const float mlo = fminf(fminf(m1, m2), fminf(m3, m4));
    const float nub = fmaf(2.0f, fabsf(fmaf(X0, Y1, -(X1 * Y0))), E);
    t2 = mloc - mlo;
    return nub * nub - thr_c * ((m1 * m2) * (m3 * m4));
}
// The same test from the fp6 screen's accumulators (pair_mfma.hip): the b
// codes read as e2m3 (F: minor 2, major 1) and as e3m2 (G: minor 2, major
// 0.5) give, in doubled units, F0 = 2T - SB, G0 = 2T - 1.5 SB (channel_a
// "in") and F1 = 2SA - SAB, G1 = 2SA - 1.5 SAB (channel_a major), so D0 =
// F0 - G0 = SB / 2, D1 = SAB / 2, and the doubled marginals of
// r2_screen_terms_xy are 2T = F0 + 2 D0, 2SB = 4 D0, 2(T - SB) = F0 - 2 D0,
// 2SA = F1 + 2 D1.  Every accumulator is an exact multiple of 1/16 below 2^19
// and R (doubled, R2) is put on that grid by the caller, so every marginal
// below, R subtracted, is exact — the xy form's marginals rounded, these equal
// the exact values.  The numerator A B - AB T = F1 D0 - F0 D1 by one product
// and one FMA: |error| <= 2u (F1 D0 + F0 D1)(1 + u) <= 4u (1 + u) T^2 of the
// doubled T, so 4 |.| is within the 4.02u Tb^2 the derivation allows (nub
// rounds once, as in the xy form).  t1 = fma(nub, nub, -fl(thr_c P)) is <= 0
// only if fl(nub^2) <= fl(thr_c P) (rounding is monotone), i.e. only where
// the xy form's t1 is <= 0.  The second test (every marginal >= mloc) is left
// to the caller as mlo (the screen tracks one minimum over a lane's pairs:
// a tile whose minimum falls below mloc is a candidate, as the xy form's t2
// would make the pair holding it).  Skip iff t1 <= 0 and mlo >= mloc.
__host__ __device__ __forceinline__ float r2_screen_terms_fg(float F0, float G0, float F1, float G1, float R2,
                                                             float thr_c, float E, float &mlo) {
    const float D0 = F0 - G0, D1 = F1 - G1;
    const float F0r = F0 - R2;
    const float m4 = fmaf(-2.0f, D0, F0r), T2r = fmaf(2.0f, D0, F0r), m3 = fmaf(4.0f, D0, -R2);
    const float A2 = fmaf(2.0f, D1, F1);
    const float m1 = A2 - R2, m2 = T2r - A2;
    mlo = fminf(fminf(m1, m2), fminf(m3, m4));
    const float nub = fmaf(4.0f, fabsf(fmaf(F1, D0, -(F0 * D1))), E);
    return fmaf(nub, nub, -(thr_c * ((m1 * m2) * (m3 * m4))));
}
// The same from the fp4-coded b sites' accumulators (pair_mfma.hip, the
// tile-pair fp6 screen with fp4 B): X = the raw codes read as e2m1 (minor 1,
// major 2), Y = their minor bit (raw & 0x2222...): X0 = T + SB, Y0 = T - SB,
// X1 = SA + SAB, Y1 = SA - SAB, so 2T = X0 + Y0, 2SB = X0 - Y0, 2(T - SB) =
// 2 Y0, 2SA = X1 + Y1 (doubled units, as r2_screen_terms_xy).  Accumulators
// and R2 on the 1/8 grid below 2^19: the marginals are exact; the numerator
// and t1 as in r2_screen_terms_xy / _fg (X0 Y1 - X1 Y0 = 2 num, error <= 2u
// (X0 Y1 + X1 Y0)(1 + u) <= 4u T^2: 2u T2^2 after doubling).  Skip iff t1 <= 0
// and mlo >= mloc.
__host__ __device__ __forceinline__ float r2_screen_terms_xy2(float X0, float Y0, float X1, float Y1, float R2,
                                                              float thr_c, float E, float &mlo) {
    const float X0r = X0 - R2;
    const float T2r = X0r + Y0, m3 = X0r - Y0, m4 = fmaf(2.0f, Y0, -R2);
    const float A2 = X1 + Y1;
    const float m1 = A2 - R2, m2 = T2r - A2;
    mlo = fminf(fminf(m1, m2), fminf(m3, m4));
    const float nub = fmaf(2.0f, fabsf(fmaf(X0, Y1, -(X1 * Y0))), E);
    return fmaf(nub, nub, -(thr_c * ((m1 * m2) * (m3 * m4))));
}
__host__ __device__ __forceinline__ float r2_screen_violation(float T, float A, float B, float AB, float R,
                                                              float thr_c) {
    float E, mloc, t2;
    screen_consts(T, R, E, mloc);
    const float t1 = r2_screen_terms(T, A, B, AB, R, thr_c, E, mloc, t2);
    return fmaxf(t1, t2);
}
__host__ __device__ __forceinline__ bool r2_screen_skip_f32(float T, float A, float B, float AB, float R, float thr) {
    return r2_screen_violation(T, A, B, AB, R, thr * (1.0f - 0x1p-7f)) <= 0.0f;
}
// largest |top-plane sum| for which the screen may use r2_screen_skip_f32
constexpr uint32_t kScreenF32MaxNP = 32768;  // 128 NP <= 2^22

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

// The same copy addressed as SGPR base + per-lane 32-bit VGPR offset (no
// 64-bit per-lane address arithmetic).
__device__ __forceinline__ void glds16_s(const void *sbase, uint32_t voff, uint32_t lds_dst) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(sbase), "s"(lds_dst)
        : "memory");
}

// ... and one dword per lane (64 lanes: 256 bytes to lds_dst + 4*lane)
__device__ __forceinline__ void glds4_s(const void *sbase, uint32_t voff, uint32_t lds_dst) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dword %1, %2\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(sbase), "s"(lds_dst)
        : "memory");
}

__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

// A tile (or part of one) of the run is finished (one thread of its
// workgroup): with per-chunk progress on, the workgroup that finishes its
// chunk's last tile appends the chunk's pair count to the host log (the value
// lib.rs's per-chunk fetch_add adds, lib.rs:670-671; the host sums the log in
// slot order).  A chunk counts kTileQuarters per tile (progress_init_kernel):
// a work item that finishes q of a tile's four 16-row blocks counts q.
constexpr uint32_t kTileQuarters = 4;
__device__ __forceinline__ void tile_done(const OrderArgs &o, uint32_t ta, uint32_t tb, uint32_t n_chunk_rows,
                                          uint32_t quarters = kTileQuarters) {
    if (!o.chunk_left) return;
    const uint32_t row = ta / kTilesPerChunk, col = tb / kTilesPerChunk;
    if (atomicSub(&o.chunk_left[chunk_linear(n_chunk_rows, row, col)], quarters) == quarters) {
        const unsigned slot = atomicAdd(o.prog_n, 1u);
        __hip_atomic_store(&o.prog_log[slot], (unsigned long long)chunk_pairs(o.L, row, col), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t t = __shfl_up(v, off, 64);
        if (lane >= off) v += t;
    }
    return v;
}

// The run's chunk scan (ScanArgs) by one workgroup of any size that is a
// multiple of 64, up to 1024: each thread sums a contiguous run of chunk
// totals, a wave scan and a scan of the wave totals give its base.  The
// counters and totals it reads were last written by other workgroups'
// agent-scope atomics in this launch (scan_tail): every load of them is an
// agent-scope (sc1) load, served past this CU's L1.
__device__ inline void chunk_scan_block(const ScanArgs &a) {
    __shared__ unsigned long long sw[16];
    auto ld32 = [](const unsigned *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    const uint32_t tid = threadIdx.x, nth = blockDim.x;
    const uint32_t per = (a.count + nth - 1) / nth;
    const uint32_t lo = min(a.count, tid * per), hi = min(a.count, lo + per);
    uint32_t *ct = a.chunk_total + a.lin_begin;
    // up to kScanRegs totals per thread (every run up to 16 x 256 chunks on a
    // 256-thread workgroup) are loaded at once, all in flight together, and
    // kept in registers for the second pass; longer runs loop
    constexpr uint32_t kScanRegs = 16;
    const bool in_regs = per <= kScanRegs;
    uint32_t vals[kScanRegs];
    unsigned long long s = 0;
    if (in_regs) {
#pragma unroll
        for (uint32_t j = 0; j < kScanRegs; ++j) vals[j] = lo + j < hi ? ld32(ct + lo + j) : 0u;
#pragma unroll
        for (uint32_t j = 0; j < kScanRegs; ++j) s += vals[j];
    } else {
        for (uint32_t i = lo; i < hi; ++i) s += ld32(ct + i);
    }
    const int lane = tid & 63, wv = tid >> 6;
    unsigned long long v = s;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const unsigned long long t = __shfl_up(v, off, 64);
        if (lane >= off) v += t;
    }
    if (lane == 63) sw[wv] = v;
    __syncthreads();
    if (tid == 0) {
        unsigned long long run = 0;
        for (uint32_t k = 0; k < nth / 64; ++k) {
            const unsigned long long t = sw[k];
            sw[k] = run;
            run += t;
        }
        *a.total = run;
        if (a.count_out) *a.count_out = run;  // e.g. the caller's tensor for the RCCL count exchange
        const unsigned long long cur = __hip_atomic_load(a.cursor, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *a.cursor = 0;
        unsigned cand = 0, blocks = 0;
        if (a.cand_count) {
            cand = ld32(a.cand_count);
            blocks = ld32(a.cand_count + 1);
        }
        // (an abandoned pass's rows are not gathered: the host re-runs it)
        if (a.cursor_seen) *a.cursor_seen = (cand & kAbandonBit) ? ~0ull : cur;
        // the next pass's candidate set starts at 0 (nothing in this launch
        // reads or writes it)
        if (a.cand_reset) a.cand_reset[0] = a.cand_reset[1] = 0;
        if (a.cand_buckets_reset)
            for (int b = 0; b < 16; ++b) a.cand_buckets_reset[b] = 0;
        if (a.host_out) {
            a.host_out[0] = cur;
            a.host_out[1] = run;
            a.host_out[2] = cand;
            a.host_out[3] = blocks;
            __threadfence_system();
        }
    }
    __syncthreads();
    unsigned long long base = sw[wv] + v - s;
    if (in_regs) {
#pragma unroll
        for (uint32_t j = 0; j < kScanRegs; ++j)
            if (lo + j < hi) {
                ct[lo + j] = 0;
                a.chunk_base[lo + j] = (uint32_t)base;
                base += vals[j];
            }
        return;
    }
    for (uint32_t i = lo; i < hi; ++i) {
        const uint32_t t = ld32(ct + i);
        ct[i] = 0;
        a.chunk_base[i] = (uint32_t)base;
        base += t;
    }
}

// The screen's candidate list in 16 buckets of capacity cap by computed 16x16
// sub-blocks (a tile with c of them in bucket 16 - c: the heaviest first, so
// the workgroups dealt round-robin over the CUs each get a mix and the list's
// light tail goes to whichever finish first); entry (b, k) at b cap + k of the
// tile and bit arrays.  The launch maps its u-th tile through the buckets'
// prefix sums, which cand_prefix puts in s_pre[17] (every thread calls it).
// An abandoned screen (kAbandonBit on bucket 0) leaves no candidate.
__device__ inline void cand_prefix(const unsigned *buckets, uint32_t *s_pre) {
    if (threadIdx.x == 0) {
        const bool abandoned = buckets[0] & kAbandonBit;
        uint32_t run = 0;
        for (int b = 0; b < 16; ++b) {
            s_pre[b] = run;
            run += abandoned ? 0u : buckets[b];
        }
        s_pre[16] = run;
    }
    __syncthreads();
}
__device__ inline uint32_t cand_entry(const uint32_t *s_pre, uint32_t cap, uint32_t u) {
    uint32_t b = 0;
    while (b < 15 && s_pre[b + 1] <= u) ++b;
    return b * cap + (u - s_pre[b]);
}
// ... guarded: ~0u (and kGuardEntry reported) unless the u-th candidate lies
// inside the buckets the screen filled (u below their total, its bucket slot
// below the capacity)
__device__ inline uint32_t cand_entry_checked(const OrderArgs &o, const uint32_t *s_pre, uint32_t cap, uint32_t u) {
    uint32_t b = 0;
    while (b < 15 && s_pre[b + 1] <= u) ++b;
    if (u >= s_pre[16] || u - s_pre[b] >= cap) {
        report_guard(o, kGuardEntry);
        return ~0u;
    }
    return b * cap + (u - s_pre[b]);
}

// The end of every workgroup of a candidate launch (a grid-stride loop over
// the screen's n_work candidate tiles).  With the scan fused (a.ticket set)
// the workgroups that computed a tile take a ticket and the last one runs the
// run's chunk scan (with no candidate, workgroup 0 alone): one launch (and
// its dispatch gap) less per run, and no ticket traffic in the common case.
// What the scan reads from this launch — the chunk totals and the staging
// cursor — is written only by agent-scope atomics (lane 63's in the
// compaction; an atomic leaves no copy of its line in the issuing XCD's L2).
// Each writing wave waits for its atomics (s_waitcnt vmcnt(0)) before lane 0
// takes the ticket; the winner then runs an agent-scope ACQUIRE (buffer_inv
// sc1: no line of the run state cached in its CU's L1 or its XCD's L2
// survives) before the scan's agent-scope loads (MI355X_MICROARCH.md,
// inter-workgroup visibility).  The acquire is the last workgroup's alone;
// no workgroup pays an L2 write-back.  WLD_OPT_FUSED_SCAN 0 runs the scan as
// a launch of its own instead (the kernel boundary orders everything).
// The screen before the launch only appended candidates (atomics, before the
// kernel boundary).
// (all_waves: every wave wrote what the scan reads, and drains before the ticket)
// first: the workgroup's first work item (a permutation of the grid's ids:
// the workgroups that computed anything are exactly those with first < p).
__device__ inline void scan_tail(const ScanArgs &a, uint32_t n_work, bool all_waves = false,
                                 uint32_t first = blockIdx.x) {
    if (!a.ticket) return;
    const uint32_t p = min(gridDim.x, n_work);  // workgroups that computed a tile
    if (first >= max(p, 1u)) return;
    __shared__ unsigned s_run;
    if (all_waves || threadIdx.x < 64) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // atomics performed
    // every wave has drained (waves that work independently may still be
    // writing when wave 0 arrives) before the workgroup takes its ticket
    if (all_waves) __syncthreads();
    if (threadIdx.x == 0) {
        s_run = p <= 1 || atomicAdd(a.ticket, 1u) == p - 1;
        if (s_run) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the invalidate completed before the barrier
        }
    }
    __syncthreads();
    if (!s_run) return;
    if (threadIdx.x == 0 && p > 1) atomicExch(a.ticket, 0u);
    chunk_scan_block(a);
}

}  // namespace wld
