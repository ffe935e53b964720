// Probe: v_mfma_scale_f32_32x32x64_f8f6f4 with fp6 e2m3 A (format 2) and fp4
// e2m1 B (format 4), unit scales.  Checks the assumed operand layout (lane l:
// A row l & 31, k = 32 (l >> 5) + j at bits 6j of six dwords; B col l & 31,
// same k, nibble j of four dwords), finds the C/D layout (which (row, col)
// each of a lane's 16 results holds) by matching against the reference
// product, and times it against the 16x16x128 form (cycles per instruction,
// one wave, 8 independent accumulators).
//   hipcc --offload-arch=gfx950 -O2 tools/probes/fp6_32_probe.hip -o /tmp/fp6_32_probe && /tmp/fp6_32_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));

__global__ void kern(const v8i *a, const v8i *b, v16f *c) {
    const int l = threadIdx.x;
    v16f acc = {};
    acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[l], b[l], acc, 2, 4, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
    c[l] = acc;
}
__global__ void rate32(const v8i *a, const v8i *b, v16f *c, long long *cyc, int n) {
    const int l = threadIdx.x;
    v8i x = a[l], y = b[l];
    v16f acc[4] = {};
    const long long t0 = clock64();
    for (int r = 0; r < n; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            acc[q] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(x, y, acc[q], 2, 4, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
    const long long t1 = clock64();
    c[l] = acc[0] + acc[1] + acc[2] + acc[3];
    if (l == 0) cyc[0] = t1 - t0;
}
__global__ void rate16(const v8i *a, const v8i *b, v4f *c, long long *cyc, int n) {
    const int l = threadIdx.x;
    v8i x = a[l], y = b[l];
    v4f acc[8] = {};
    const long long t0 = clock64();
    for (int r = 0; r < n; ++r)
#pragma unroll
        for (int q = 0; q < 8; ++q)
            acc[q] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(x, y, acc[q], 2, 4, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
    const long long t1 = clock64();
    v4f s = acc[0];
    for (int q = 1; q < 8; ++q) s += acc[q];
    c[l] = s;
    if (l == 0) cyc[0] = t1 - t0;
}

static float fp4(unsigned c) {
    const float mag[8] = {0.f, 0.5f, 1.f, 1.5f, 2.f, 3.f, 4.f, 6.f};
    return (c & 8) ? -mag[c & 7] : mag[c & 7];
}
static float fp6(unsigned c) {
    const unsigned e = (c >> 3) & 3, m = c & 7;
    const float v = e ? (1.0f + m / 8.0f) * (float)(1 << (e - 1)) : m / 8.0f;
    return (c & 32) ? -v : v;
}

int main() {
    v8i ha[64], hb[64];
    static float A[32][64], B[64][32];
    srand(7);
    memset(ha, 0, sizeof ha);
    memset(hb, 0, sizeof hb);
    for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 32; ++j) {
            const unsigned ca = rand() & 63, cb = (unsigned[]){0, 2, 4, 3, 1}[rand() % 5];
            const int bit = 6 * j;
            ha[l][bit / 32] |= (int)(ca << (bit % 32));
            if (bit % 32 > 26) ha[l][bit / 32 + 1] |= (int)(ca >> (32 - bit % 32));
            hb[l][j / 8] |= (int)(cb << (4 * (j % 8)));
            A[l & 31][32 * (l >> 5) + j] = fp6(ca);
            B[32 * (l >> 5) + j][l & 31] = fp4(cb);
        }
    double ref[32][32];
    for (int r = 0; r < 32; ++r)
        for (int c = 0; c < 32; ++c) {
            double s = 0;
            for (int k = 0; k < 64; ++k) s += (double)A[r][k] * B[k][c];
            ref[r][c] = s;
        }
    v8i *da, *db;
    v16f *dc;
    long long *dcyc;
    hipMalloc(&da, sizeof ha);
    hipMalloc(&db, sizeof hb);
    hipMalloc(&dc, 64 * sizeof(v16f));
    hipMalloc(&dcyc, sizeof(long long));
    hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, da, db, dc);
    v16f hc[64];
    hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost);
    // the assumed C/D layout: col = l & 31, row = 8 (i / 4) + 4 (l / 32) + i % 4
    int bad = 0, ambiguous = 0;
    for (int l = 0; l < 64; ++l)
        for (int i = 0; i < 16; ++i) {
            const int row = 8 * (i / 4) + 4 * (l / 32) + i % 4, col = l & 31;
            if ((double)hc[l][i] != ref[row][col]) {
                if (bad < 6) {
                    printf("layout mismatch lane %d i %d: gpu %.4f expected (%d,%d) %.4f; matches:", l, i, hc[l][i], row,
                           col, ref[row][col]);
                    int n = 0;
                    for (int r = 0; r < 32; ++r)
                        for (int c = 0; c < 32; ++c)
                            if (ref[r][c] == (double)hc[l][i] && n++ < 4) printf(" (%d,%d)", r, c);
                    printf("\n");
                }
                ++bad;
            }
        }
    (void)ambiguous;
    printf("fp6 x fp4 32x32x64 layout (A/B as assumed, C/D row = 8(i/4) + 4(l/32) + i%%4, col = l&31): %s (%d mismatches)\n",
           bad ? "FAIL" : "ok", bad);
    const int n = 256;
    long long cyc[2];
    hipLaunchKernelGGL(rate32, dim3(1), dim3(64), 0, 0, da, db, dc, dcyc, n);
    hipMemcpy(&cyc[0], dcyc, sizeof(long long), hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(rate16, dim3(1), dim3(64), 0, 0, da, db, (v4f *)dc, dcyc, n);
    hipMemcpy(&cyc[1], dcyc, sizeof(long long), hipMemcpyDeviceToHost);
    printf("cycles per MFMA (one wave): 32x32x64 %.2f (4 accumulators), 16x16x128 %.2f (8 accumulators); per "
           "16x16x128-equivalent: %.2f vs %.2f\n",
           (double)cyc[0] / (4.0 * n), (double)cyc[1] / (8.0 * n), (double)cyc[0] / (8.0 * n),
           (double)cyc[1] / (8.0 * n));
    return bad != 0;
}
