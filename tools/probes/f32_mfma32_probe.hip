// f32 MFMA shape probe: cycles per 1,024 MACs per SIMD (s_memtime) for
// v_mfma_f32_16x16x4_f32 (1,024 MACs) against v_mfma_f32_32x32x2_f32 (2,048),
// with 1 / 2 / 4 / 8 waves per SIMD, for
//   dep      four accumulators round robin, operands in registers
//   shared   the item kernel's full-run pattern: A operands (u, v) read from
//            LDS as one float2, B formed by two byte converts, four MFMAs
//            (one per channel pair) per element
// One workgroup of 4 waves per SIMD-wave slot group (W workgroups per CU).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));

template <int MODE>
__global__ __launch_bounds__(256) void probe(float *out, unsigned long long *cyc, int iters, unsigned seed) {
    __shared__ float2 sA[1024];
    const unsigned lane = threadIdx.x & 63;
    for (unsigned i = threadIdx.x; i < 1024; i += 256) sA[i] = make_float2(1.0f + i * 1e-3f, 0.5f);
    __syncthreads();
    float a = 1.0f + lane * 1e-3f, b = 0.5f + (seed & 7);
    unsigned code = 0x01000101u * (lane + seed);
    constexpr bool k32 = MODE == 1 || MODE == 3;
    v4f acc[4];
    v16f acc32[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc32[q][j] = 0.f;
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < iters; ++it) {
        if constexpr (MODE == 0) {  // dep, 16x16x4: 16 MFMAs
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[q], 0, 0, 0);
        } else if constexpr (MODE == 1) {  // dep, 32x32x2: 16 MFMAs
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    acc32[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc32[q], 0, 0, 0);
        } else {  // shared pattern: 16 MFMAs
            const unsigned bi = code & 0x01010101u, bm = (code >> 1) & 0x01010101u;
            const float2 *src = sA + ((it * 64 + lane) & 1023);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float2 uv = src[(64 * e) & 1023];
                const float fi = (float)((bi >> (8 * e)) & 0xFFu), fm = (float)((bm >> (8 * e)) & 0xFFu);
                if constexpr (k32) {
                    acc32[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(uv.x, fi, acc32[0], 0, 0, 0);
                    acc32[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(uv.y, fi, acc32[1], 0, 0, 0);
                    acc32[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(uv.x, fm, acc32[2], 0, 0, 0);
                    acc32[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(uv.y, fm, acc32[3], 0, 0, 0);
                } else {
                    acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(uv.x, fi, acc[0], 0, 0, 0);
                    acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(uv.y, fi, acc[1], 0, 0, 0);
                    acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(uv.x, fm, acc[2], 0, 0, 0);
                    acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(uv.y, fm, acc[3], 0, 0, 0);
                }
            }
            code = code * 1664525u + 1013904223u;
        }
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        s += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
#pragma unroll
        for (int j = 0; j < 16; ++j) s += acc32[q][j];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (lane == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int MODE>
double run(int W, int iters) {
    const int blocks = 256 * W, threads = 256;
    float *out;
    unsigned long long *cyc;
    if (hipMalloc(&out, (size_t)blocks * threads * 4) || hipMalloc(&cyc, (size_t)blocks * threads / 64 * 8)) return -1;
    hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters / 4, 1u);  // warm
    hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters, 1u);
    if (hipDeviceSynchronize()) return -2;
    std::vector<unsigned long long> h((size_t)blocks * threads / 64);
    hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
    double mean = 0;
    for (auto v : h) mean += (double)v;
    mean /= h.size();
    hipFree(out);
    hipFree(cyc);
    const double macs = (MODE == 1 || MODE == 3) ? 2.0 : 1.0;  // per MFMA, in units of 1,024
    return mean / (16.0 * iters * W * macs);
}

int main() {
    for (int W : {1, 2, 3, 4, 8}) {  // (the 32x32 modes hold 3 waves per SIMD at most)
        const double d16 = run<0>(W, 2000), d32 = run<1>(W, 2000), s16 = run<2>(W, 2000), s32 = run<3>(W, 2000);
        printf("waves/SIMD %d: cycles per 1024 MACs per SIMD  dep16 %.1f  dep32 %.1f  shared16 %.1f  shared32 %.1f\n", W,
               d16, d32, s16, s32);
    }
    return 0;
}
