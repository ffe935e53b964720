// Probe: does passing zero scale operands to the f8f6f4 MFMA builtin (which
// the compiler lowers to the unscaled v_mfma_f32_16x16x128_f8f6f4) give the
// same sums as the unit-scaled v_mfma_scale form the fp6 screen uses (fp6
// e2m3 A, fp4 e2m1 B), and at what issue rate (cycles per instruction per
// SIMD, eight independent accumulators, 1-3 waves per SIMD)?
//   hipcc --offload-arch=gfx950 -O2 tools/probes/fp6_unscaled_probe.hip -o /tmp/p && /tmp/p
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

template <bool UNSCALED>
__device__ __forceinline__ v4f mf(v8i a, v8i b, v4f c) {
    if constexpr (UNSCALED)
        return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 2, 4, 0, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 2, 4, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
}

template <bool UNSCALED>
__global__ void sums(const v8i *a, const v8i *b, v4f *c, int reps) {
    const int l = threadIdx.x;
    v4f acc = {0, 0, 0, 0};
    for (int r = 0; r < reps; ++r) acc = mf<UNSCALED>(a[64 * r + l], b[64 * r + l], acc);
    c[l] = acc;
}

template <bool UNSCALED>
__global__ void rate(const v8i *a, const v8i *b, v4f *c, long long *cyc, int n) {
    const int l = threadIdx.x & 63;
    v8i x = a[l], y = b[l];
    v4f acc[8] = {};
    __syncthreads();
    const long long t0 = clock64();
    for (int r = 0; r < n; ++r)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] = mf<UNSCALED>(x, y, acc[q]);
    const long long t1 = clock64();
    v4f s = acc[0];
    for (int q = 1; q < 8; ++q) s += acc[q];
    c[threadIdx.x] = s;
    if (l == 0) cyc[threadIdx.x / 64] = t1 - t0;
}

int main() {
    const int reps = 64, n = 2048;
    v8i *ha = (v8i *)malloc(sizeof(v8i) * 64 * reps), *hb = (v8i *)malloc(sizeof(v8i) * 64 * reps);
    srand(7);
    for (int i = 0; i < 64 * reps; ++i)
        for (int j = 0; j < 8; ++j) {
            ha[i][j] = j < 6 ? rand() ^ (rand() << 16) : 0;
            // fp4 B: nibbles 0, 2 (1.0) or 4 (2.0), as the screen's codes
            unsigned v = 0;
            for (int q = 0; q < 8; ++q) v |= (unsigned)((rand() % 3) * 2) << (4 * q);
            hb[i][j] = j < 4 ? (int)v : 0;
        }
    v8i *da, *db;
    v4f *dc;
    long long *dcyc;
    hipMalloc(&da, sizeof(v8i) * 64 * reps);
    hipMalloc(&db, sizeof(v8i) * 64 * reps);
    hipMalloc(&dc, sizeof(v4f) * 64 * 16);
    hipMalloc(&dcyc, sizeof(long long) * 16);
    hipMemcpy(da, ha, sizeof(v8i) * 64 * reps, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, sizeof(v8i) * 64 * reps, hipMemcpyHostToDevice);
    v4f r0[64], r1[64];
    hipLaunchKernelGGL(sums<false>, dim3(1), dim3(64), 0, 0, da, db, dc, reps);
    hipMemcpy(r0, dc, sizeof(r0), hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(sums<true>, dim3(1), dim3(64), 0, 0, da, db, dc, reps);
    hipMemcpy(r1, dc, sizeof(r1), hipMemcpyDeviceToHost);
    int diff = 0;
    double mag = 0;
    for (int l = 0; l < 64; ++l)
        for (int e = 0; e < 4; ++e) {
            diff += r0[l][e] != r1[l][e];
            mag += fabs(r0[l][e]);
        }
    printf("unscaled vs unit-scaled sums: %d of 256 differ (mean |sum| %.3f; sample %.4f vs %.4f)\n", diff, mag / 256,
           r0[5][1], r1[5][1]);
    for (int w = 1; w <= 3; ++w)
        for (int u = 0; u < 2; ++u) {
            long long cyc[16];
            // one workgroup of 4w waves: w waves per SIMD
            if (u)
                hipLaunchKernelGGL(rate<true>, dim3(1), dim3(256 * w), 0, 0, da, db, dc, dcyc, n);
            else
                hipLaunchKernelGGL(rate<false>, dim3(1), dim3(256 * w), 0, 0, da, db, dc, dcyc, n);
            hipMemcpy(cyc, dcyc, sizeof(long long) * 4 * w, hipMemcpyDeviceToHost);
            double mx = 0;
            for (int i = 0; i < 4 * w; ++i) mx = cyc[i] > mx ? cyc[i] : mx;
            printf("%s, %d wave(s) per SIMD: %.2f cycles per MFMA per SIMD (clock64 units)\n",
                   u ? "unscaled" : "unit-scaled", w, mx / (8.0 * n * w));
        }
    return diff != 0;
}
