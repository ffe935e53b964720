// f32 MFMA 32x32x2 in "quadrant" form for lib.rs's ordered sums: rows 0-15
// of A = w x in(a site), rows 16-31 = w x major(a site); columns 0-15 of B =
// in(b site), 16-31 = major(b site); k = two consecutive sequences.  One
// instruction then gives all four sums of 16 x 16 site pairs over two
// sequences in ONE 16-register accumulator (the 16x16x4 form needs four).
//
// Part 1 (exactness): a chain of T instructions on one accumulator against
// host models of the per-element order: k0 then k1 with an f32 rounding after
// each add (lib.rs's in-order chain), k1 then k0, and one rounding of
// acc + p0 + p1.  Products are exact (B is 0/1).  Also checks the output
// layout assumed below (lane l: column l % 32, register i: row 8 (i / 4) +
// 4 (l / 32) + i % 4).
// Part 2 (rate): cycles per 1,024 MACs per SIMD at 1..8 waves per SIMD for
//   s16   the item kernel's pattern today: A (u, v) as one float2 from LDS,
//         two byte converts for B, four 16x16x4 MFMAs per sequence group
//   q32   quadrant form: A as one float from LDS per instruction, B one byte
//         convert of the lane's channel bit, two 32x32x2 per 4 sequences on
//         ONE accumulator (a dependent chain)
//   q32x2 the same on two accumulators alternating (two class chains
//         interleaved)
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(64) void exact32(const float *A, const float *B, int T, float *D) {
    const unsigned l = threadIdx.x;
    v16f acc;
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    for (int t = 0; t < T; ++t) {
        const float a = A[(size_t)t * 64 + (l % 32) * 2 + l / 32];  // A[t][m][k]
        const float b = B[(size_t)t * 64 + (l / 32) * 32 + l % 32];  // B[t][k][n]
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    for (int i = 0; i < 16; ++i) {
        const unsigned m = 8 * (i / 4) + 4 * (l / 32) + i % 4, n = l % 32;
        D[m * 32 + n] = acc[i];
    }
}

template <int MODE>
__global__ __launch_bounds__(256) void rate(float *out, unsigned long long *cyc, int iters, unsigned seed) {
    __shared__ float2 sA[1024];
    const unsigned lane = threadIdx.x & 63;
    for (unsigned i = threadIdx.x; i < 1024; i += 256) sA[i] = make_float2(1.0f + i * 1e-3f, 0.5f);
    __syncthreads();
    unsigned code = 0x01000101u * (lane + seed);
    const unsigned chs = (lane >> 4) & 1u;  // q32: the lane's channel bit (in / major)
    v4f acc[4];
    v16f q0, q1;
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 16; ++j) q0[j] = q1[j] = 0.f;
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < iters; ++it) {
        const float2 *src = sA + ((it * 64 + lane) & 1023);
        if constexpr (MODE == 0) {  // s16: 16 MFMAs of 1,024 MACs
            const unsigned bi = code & 0x01010101u, bm = (code >> 1) & 0x01010101u;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float2 uv = src[(64 * e) & 1023];
                const float fi = (float)((bi >> (8 * e)) & 0xFFu), fm = (float)((bm >> (8 * e)) & 0xFFu);
                acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(uv.x, fi, acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(uv.y, fi, acc[1], 0, 0, 0);
                acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(uv.x, fm, acc[2], 0, 0, 0);
                acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(uv.y, fm, acc[3], 0, 0, 0);
            }
        } else {  // q32 / q32x2: 8 MFMAs of 2,048 MACs (the same 16,384 MACs)
            const unsigned bsel = (code >> chs) & 0x01010101u;
            const float *srcf = reinterpret_cast<const float *>(src);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float fb = (float)((bsel >> (8 * e)) & 0xFFu);
                const float a0 = srcf[(128 * e) & 2047], a1 = srcf[(128 * e + 64) & 2047];
                if constexpr (MODE == 1) {
                    q0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, fb, q0, 0, 0, 0);
                    q0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, fb, q0, 0, 0, 0);
                } else {
                    q0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, fb, q0, 0, 0, 0);
                    q1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, fb, q1, 0, 0, 0);
                }
            }
        }
        code = code * 1664525u + 1013904223u;
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) s += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
#pragma unroll
    for (int j = 0; j < 16; ++j) s += q0[j] + q1[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (lane == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int MODE>
double run(int W, int iters) {
    const int blocks = 256 * W, threads = 256;
    float *out;
    unsigned long long *cyc;
    if (hipMalloc(&out, (size_t)blocks * threads * 4) || hipMalloc(&cyc, (size_t)blocks * threads / 64 * 8)) return -1;
    hipLaunchKernelGGL(rate<MODE>, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters / 4, 1u);  // warm
    hipLaunchKernelGGL(rate<MODE>, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters, 1u);
    if (hipDeviceSynchronize()) return -2;
    std::vector<unsigned long long> h((size_t)blocks * threads / 64);
    hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
    double mean = 0;
    for (auto v : h) mean += (double)v;
    mean /= h.size();
    hipFree(out);
    hipFree(cyc);
    return mean / (16.0 * iters * W);  // every mode: 16 x 1,024 MACs per iteration
}

static unsigned long long rng = 88172645463325252ull;
static unsigned nxt() {
    rng ^= rng << 13, rng ^= rng >> 7, rng ^= rng << 17;
    return (unsigned)(rng >> 11);
}

int main() {
    // ---- part 1: exactness -------------------------------------------------
    const int T = 512;
    std::vector<float> A((size_t)T * 64), B((size_t)T * 64), D(1024);
    for (int pass = 0; pass < 2; ++pass) {
        for (auto &a : A) {  // wide exponents so that the add order shows in the last bits
            const int ex = pass == 0 ? 0 : (int)(nxt() % 41) - 20;
            a = std::ldexp(1.0f + (nxt() % (1u << 23)) / (float)(1u << 23), ex) * ((nxt() & 1) ? -1.f : 1.f);
            if (pass == 0) a = std::fabs(a) * 0.01f;
        }
        for (auto &b : B) b = (nxt() % 10) < 7 ? 1.0f : 0.0f;
        float *dA, *dB, *dD;
        hipMalloc(&dA, A.size() * 4), hipMalloc(&dB, B.size() * 4), hipMalloc(&dD, 4096);
        hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
        hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
        // layout check on one instruction (exact in double)
        hipLaunchKernelGGL(exact32, dim3(1), dim3(64), 0, 0, dA, dB, 1, dD);
        hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost);
        int lay_bad = 0;
        for (int m = 0; m < 32; ++m)
            for (int n = 0; n < 32; ++n) {
                const double r = (double)A[m * 2] * B[n] + (double)A[m * 2 + 1] * B[32 + n];
                if (std::fabs(r - D[m * 32 + n]) > 1e-6 * (std::fabs(r) + 1e-30) + 1e-38) ++lay_bad;
            }
        hipLaunchKernelGGL(exact32, dim3(1), dim3(64), 0, 0, dA, dB, T, dD);
        hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost);
        int ok01 = 0, ok10 = 0, ok1r = 0, okpair = 0;
        for (int m = 0; m < 32; ++m)
            for (int n = 0; n < 32; ++n) {
                float s01 = 0.f, s10 = 0.f, s1r = 0.f, sp = 0.f;
                for (int t = 0; t < T; ++t) {
                    const float p0 = A[(size_t)t * 64 + m * 2] * B[(size_t)t * 64 + n];
                    const float p1 = A[(size_t)t * 64 + m * 2 + 1] * B[(size_t)t * 64 + 32 + n];
                    volatile float x = s01 + p0;
                    s01 = x + p1;
                    volatile float y = s10 + p1;
                    s10 = y + p0;
                    s1r = (float)((double)s1r + (double)p0 + (double)p1);
                    volatile float z = p0 + p1;
                    sp = sp + z;
                }
                const float g = D[m * 32 + n];
                ok01 += !memcmp(&g, &s01, 4);
                ok10 += !memcmp(&g, &s10, 4);
                ok1r += !memcmp(&g, &s1r, 4);
                okpair += !memcmp(&g, &sp, 4);
            }
        printf("exactness (%s exponents, T=%d, 1024 sums): layout mismatches %d; equal to k0-then-k1 %d, "
               "k1-then-k0 %d, one rounding %d, (p0+p1) then acc %d\n",
               pass == 0 ? "narrow" : "wide", T, lay_bad, ok01, ok10, ok1r, okpair);
        hipFree(dA), hipFree(dB), hipFree(dD);
    }
    // ---- part 2: rate ------------------------------------------------------
    for (int W : {1, 2, 3, 4, 6, 8}) {
        const double s16 = run<0>(W, 2000), q32 = run<1>(W, 2000), q32x2 = run<2>(W, 2000);
        printf("waves/SIMD %d: cycles per 1024 MACs per SIMD  s16 %.1f  q32 %.1f  q32x2 %.1f\n", W, s16, q32, q32x2);
    }
    return 0;
}
