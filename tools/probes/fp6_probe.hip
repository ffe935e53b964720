// Probe: v_mfma_scale_f32_16x16x128_f8f6f4 with fp6 e2m3 A (format 2) and fp4
// e2m1 B (format 4), unit scales.  Checks (1) the fp6 operand packing: lane l
// holds A[row l&15][k = 32 (l>>4) + j], element j at bits [6j, 6j+6) of its
// six dwords; fp4: B[k = 32 (l>>4) + j][col l&15], nibble j of four dwords
// (tools/probes/fp4_probe.hip), (2) that the f32 sums of products of fp6 x fp4
// values are exact (multiples of 1/16, far below 2^24 units), (3) the C/D
// layout (col = lane & 15, row = 4 (lane >> 4) + e), and (4) the issue rate of
// the mixed fp6 x fp4 form against i8 16x16x64 (cycles per instruction).
//   hipcc --offload-arch=gfx950 -O2 tools/probes/fp6_probe.hip -o /tmp/fp6_probe && /tmp/fp6_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));

template <int FA, int FB>
__global__ void kern(const v8i *a, const v8i *b, v4f *c, int reps) {
    const int l = threadIdx.x;
    v4f acc = {0, 0, 0, 0};
    for (int r = 0; r < reps; ++r)
        acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], acc, FA, FB, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
    c[l] = acc;
}

// rate: 8 independent accumulators, n instructions each, per wave; clock64 around
template <int FA, int FB>
__global__ void rate(const v8i *a, const v8i *b, v4f *c, long long *cyc, int n) {
    const int l = threadIdx.x;
    v8i x = a[l], y = b[l];
    v4f acc[8] = {};
    const long long t0 = clock64();
    for (int r = 0; r < n; ++r)
#pragma unroll
        for (int q = 0; q < 8; ++q)
            acc[q] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(x, y, acc[q], FA, FB, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
    const long long t1 = clock64();
    v4f s = acc[0];
    for (int q = 1; q < 8; ++q) s += acc[q];
    c[l] = s;
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}
__global__ void rate_i8(const v8i *a, const v8i *b, v4f *c, long long *cyc, int n) {
    const int l = threadIdx.x;
    v4i x = {a[l][0], a[l][1], a[l][2], a[l][3]}, y = {b[l][0], b[l][1], b[l][2], b[l][3]};
    v4i acc[8] = {};
    const long long t0 = clock64();
    for (int r = 0; r < n; ++r)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] = __builtin_amdgcn_mfma_i32_16x16x64_i8(x, y, acc[q], 0, 0, 0);
    const long long t1 = clock64();
    v4i s = acc[0];
    for (int q = 1; q < 8; ++q) s += acc[q];
    c[l] = v4f{(float)s[0], (float)s[1], (float)s[2], (float)s[3]};
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

static float fp4(unsigned c) {
    const float mag[8] = {0.f, 0.5f, 1.f, 1.5f, 2.f, 3.f, 4.f, 6.f};
    return (c & 8) ? -mag[c & 7] : mag[c & 7];
}
// e2m3: sign, 2 exponent bits (bias 1), 3 mantissa bits; subnormal at exponent 0
static float fp6(unsigned c) {
    const unsigned e = (c >> 3) & 3, m = c & 7;
    const float v = e ? (1.0f + m / 8.0f) * (float)(1 << (e - 1)) : m / 8.0f;
    return (c & 32) ? -v : v;
}

int main() {
    v8i ha[64], hb[64];
    static float A[16][128], B[128][16];
    srand(11);
    memset(ha, 0, sizeof ha);
    memset(hb, 0, sizeof hb);
    for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 32; ++j) {
            const unsigned ca = rand() & 63, cb = (unsigned[]){0, 2, 4, 3}[rand() % 4];
            const int bit = 6 * j;
            ha[l][bit / 32] |= (int)(ca << (bit % 32));
            if (bit % 32 > 26) ha[l][bit / 32 + 1] |= (int)(ca >> (32 - bit % 32));
            hb[l][j / 8] |= (int)(cb << (4 * (j % 8)));
            A[l & 15][32 * (l >> 4) + j] = fp6(ca);
            B[32 * (l >> 4) + j][l & 15] = fp4(cb);
        }
    v8i *da, *db;
    v4f *dc;
    long long *dcyc;
    hipMalloc(&da, sizeof ha);
    hipMalloc(&db, sizeof hb);
    hipMalloc(&dc, 64 * sizeof(v4f));
    hipMalloc(&dcyc, 64 * sizeof(long long));
    hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
    int bad = 0;
    for (int reps : {1, 9}) {
        hipLaunchKernelGGL((kern<2, 4>), dim3(1), dim3(64), 0, 0, da, db, dc, reps);
        v4f hc[64];
        hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost);
        for (int l = 0; l < 64; ++l)
            for (int e = 0; e < 4; ++e) {
                const int row = 4 * (l >> 4) + e, col = l & 15;
                double ref = 0;
                for (int k = 0; k < 128; ++k) ref += (double)A[row][k] * B[k][col];
                ref *= reps;
                if ((double)hc[l][e] != ref) {
                    if (bad < 8) printf("mismatch reps %d row %d col %d: gpu %.5f ref %.5f\n", reps, row, col, hc[l][e], ref);
                    ++bad;
                }
            }
    }
    printf("fp6 x fp4 layout/exactness: %s (%d mismatches)\n", bad ? "FAIL" : "ok", bad);
    long long cyc[2];
    const int n = 512;
    hipLaunchKernelGGL((rate<2, 4>), dim3(1), dim3(64), 0, 0, da, db, dc, dcyc, n);
    hipMemcpy(&cyc[0], dcyc, sizeof(long long), hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(rate_i8, dim3(1), dim3(64), 0, 0, da, db, dc, dcyc, n);
    hipMemcpy(&cyc[1], dcyc, sizeof(long long), hipMemcpyDeviceToHost);
    printf("cycles per MFMA (one wave, 8 accumulators): fp6xfp4 16x16x128 %.2f, i8 16x16x64 %.2f\n",
           (double)cyc[0] / (8.0 * n), (double)cyc[1] / (8.0 * n));
    return bad != 0;
}
