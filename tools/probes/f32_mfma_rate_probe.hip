// f32 MFMA issue-rate probe (v_mfma_f32_16x16x4_f32): cycles per MFMA per
// SIMD with W waves per SIMD (1, 2, 4, 8), for
//   dep4   4 accumulators round robin, operands in registers (no VALU)
//   dep8   8 accumulators round robin
//   item   the item kernel's pattern: per element two byte converts and two
//          multiplies for the A side, two converts for the B side, then the
//          four MFMAs (operands formed from registers, no memory)
// W workgroups of 4 waves per CU (W waves per SIMD), 256 CUs; s_memtime
// around the loop in each wave; reports the mean over waves of (cycles / MFMAs
// per SIMD), i.e. cycles per MFMA per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float v4f __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void probe(float *out, unsigned long long *cyc, int iters, unsigned seed) {
    const unsigned lane = threadIdx.x & 63;
    float a = 1.0f + lane * 1e-3f, b = 0.5f + (seed & 7);
    unsigned code = 0x01000101u * (lane + seed);
    v4f acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = v4f{0.f, 0.f, 0.f, 0.f};
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < iters; ++it) {
        if constexpr (MODE == 0) {  // dep4: 16 MFMAs
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[q], 0, 0, 0);
        } else if constexpr (MODE == 1) {  // dep8: 16 MFMAs
#pragma unroll
            for (int e = 0; e < 2; ++e)
#pragma unroll
                for (int q = 0; q < 8; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[q], 0, 0, 0);
        } else {  // item pattern: 16 MFMAs
            const unsigned ai = code & 0x01010101u, am = (code >> 1) & 0x01010101u;
            const unsigned bi = (code >> 2) & 0x01010101u, bm = (code >> 3) & 0x01010101u;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float u = a * (float)((ai >> (8 * e)) & 0xFFu), v = a * (float)((am >> (8 * e)) & 0xFFu);
                const float fi = (float)((bi >> (8 * e)) & 0xFFu), fm = (float)((bm >> (8 * e)) & 0xFFu);
                acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(u, fi, acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(v, fi, acc[1], 0, 0, 0);
                acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(u, fm, acc[2], 0, 0, 0);
                acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(v, fm, acc[3], 0, 0, 0);
            }
            code = code * 1664525u + 1013904223u;
        }
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) s += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (lane == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int MODE>
double run(int W, int iters) {
    const int blocks = 256 * W, threads = 256;  // W workgroups of 4 waves per CU: W waves per SIMD
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
    // each wave did 16 * iters MFMAs; W waves share a SIMD
    return mean / (16.0 * iters * W);
}

int main() {
    const char *names[3] = {"dep4", "dep8", "item"};
    for (int W : {1, 2, 4, 8}) {
        double r0 = run<0>(W, 2000), r1 = run<1>(W, 2000), r2 = run<2>(W, 2000);
        printf("waves/SIMD %d: cycles per MFMA per SIMD  %s %.1f  %s %.1f  %s %.1f\n", W, names[0], r0, names[1], r1,
               names[2], r2);
    }
    return 0;
}
