// Probe: v_mfma_scale_f32_16x16x128_f8f6f4 and _32x32x64_ with fp4 (e2m1) A
// and B, unit scales.  Checks (1) that A lane (row l&15, group l>>4, nibble e)
// and B lane (col l&15, group l>>4, nibble e) multiply the same k (32x32x64:
// row/col l&31, group l>>5), (2) that the f32 sums of products of fp4 values
// are exact (multiples of 0.25, |sum| < 2^20), (3) the C/D layouts.
//   hipcc --offload-arch=gfx950 -O2 tools/probes/fp4_probe.hip -o /tmp/fp4_probe && /tmp/fp4_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

typedef float v16f __attribute__((ext_vector_type(16)));
__global__ void kern32(const v8i *a, const v8i *b, v16f *c, int reps) {
    const int l = threadIdx.x;
    v16f acc = {};
    for (int r = 0; r < reps; ++r)
        acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[l], b[l], acc, 4, 4, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
    c[l] = acc;
}

__global__ void kern(const v8i *a, const v8i *b, v4f *c, int reps) {
    const int l = threadIdx.x;
    v4f acc = {0, 0, 0, 0};
    for (int r = 0; r < reps; ++r)
        acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], acc, 4, 4, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
    c[l] = acc;
}

static float fp4(unsigned c) {
    const float mag[8] = {0.f, 0.5f, 1.f, 1.5f, 2.f, 3.f, 4.f, 6.f};
    return (c & 8) ? -mag[c & 7] : mag[c & 7];
}

int main() {
    v8i ha[64], hb[64];
    float A[16][128], B[128][16];
    srand(7);
    memset(ha, 0, sizeof ha);
    memset(hb, 0, sizeof hb);
    for (int l = 0; l < 64; ++l)
        for (int e = 0; e < 32; ++e) {
            const unsigned ca = rand() & 15, cb = (unsigned[]){0, 2, 4}[rand() % 3];
            ha[l][e / 8] |= (int)(ca << (4 * (e % 8)));
            hb[l][e / 8] |= (int)(cb << (4 * (e % 8)));
            A[l & 15][32 * (l >> 4) + e] = fp4(ca);
            B[32 * (l >> 4) + e][l & 15] = fp4(cb);
        }
    v8i *da, *db;
    v4f *dc;
    hipMalloc(&da, sizeof ha);
    hipMalloc(&db, sizeof hb);
    hipMalloc(&dc, 64 * sizeof(v4f));
    hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
    int bad = 0;
    for (int reps : {1, 7}) {
        hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, da, db, dc, reps);
        v4f hc[64];
        hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost);
        for (int l = 0; l < 64; ++l)
            for (int e = 0; e < 4; ++e) {
                const int row = 4 * (l >> 4) + e, col = l & 15;  // C/D layout of 16x16 MFMAs
                double ref = 0;
                for (int k = 0; k < 128; ++k) ref += (double)A[row][k] * B[k][col];
                ref *= reps;
                if ((double)hc[l][e] != ref) {
                    if (bad < 8) printf("mismatch reps %d row %d col %d: gpu %.4f ref %.4f\n", reps, row, col, hc[l][e], ref);
                    ++bad;
                }
            }
    }
    // 32x32x64: lane l: A[row l&31][k = 32 (l>>5) + e], B[k][col l&31]
    float A2[32][64], B2[64][32];
    memset(ha, 0, sizeof ha);
    memset(hb, 0, sizeof hb);
    for (int l = 0; l < 64; ++l)
        for (int e = 0; e < 32; ++e) {
            const unsigned ca = rand() & 15, cb = (unsigned[]){0, 2, 4}[rand() % 3];
            ha[l][e / 8] |= (int)(ca << (4 * (e % 8)));
            hb[l][e / 8] |= (int)(cb << (4 * (e % 8)));
            A2[l & 31][32 * (l >> 5) + e] = fp4(ca);
            B2[32 * (l >> 5) + e][l & 31] = fp4(cb);
        }
    hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
    v16f *dc2;
    hipMalloc(&dc2, 64 * sizeof(v16f));
    for (int reps : {1, 5}) {
        hipLaunchKernelGGL(kern32, dim3(1), dim3(64), 0, 0, da, db, dc2, reps);
        v16f hc[64];
        hipMemcpy(hc, dc2, sizeof hc, hipMemcpyDeviceToHost);
        for (int l = 0; l < 64; ++l)
            for (int i = 0; i < 16; ++i) {
                const int row = (i & 3) + 8 * (i >> 2) + 4 * (l >> 5), col = l & 31;
                double ref = 0;
                for (int k = 0; k < 64; ++k) ref += (double)A2[row][k] * B2[k][col];
                ref *= reps;
                if ((double)hc[l][i] != ref) {
                    if (bad < 16) printf("32x32 mismatch reps %d row %d col %d: gpu %.4f ref %.4f\n", reps, row, col, hc[l][i], ref);
                    ++bad;
                }
            }
    }
    printf("fp4 probe: %s (%d mismatches)\n", bad ? "FAIL" : "ok", bad);
    return bad != 0;
}
