// Probe: one 6-bit B operand read two ways by v_mfma_scale_f32_16x16x128_f8f6f4
// (blgp 2 = fp6 e2m3, blgp 3 = bf6 e3m2), A fp6 e2m3 (cbsz 2), unit scales.
// The fp6 screen (pair_mfma.hip) codes a b site's symbol as 0 (neither major
// nor minor), 8 (major) or 16 (minor): e2m3 reads them as 0 / 1.0 / 2.0 and
// e3m2 as 0 / 0.5 / 2.0, so the two readings of the same bytes are two
// independent channels with no mask instruction.  Checks (1) those decodings
// and the fp6 packing of B (lane l holds B[k = 32 (l>>4) + j][col l&15] at
// bits 6j of six dwords, as A), (2) exact f32 sums, (3) the C/D layout, and
// (4) cycles per instruction of fp6 x fp6 and fp6 x bf6 against fp6 x fp4.
//   hipcc --offload-arch=gfx950 -O2 tools/probes/fp6_dual_probe.hip -o /tmp/fp6_dual_probe && /tmp/fp6_dual_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

template <int FA, int FB>
__global__ void kern(const v8i *a, const v8i *b, v4f *c) {
    const int l = threadIdx.x;
    c[l] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], v4f{0, 0, 0, 0}, FA, FB, 0, 0x7F7F7F7F, 0,
                                                            0x7F7F7F7F);
}

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

static float e2m3(unsigned c) {
    const unsigned e = (c >> 3) & 3, m = c & 7;
    const float v = e ? (1.0f + m / 8.0f) * (float)(1 << (e - 1)) : m / 8.0f;
    return (c & 32) ? -v : v;
}
static float e3m2(unsigned c) {
    const unsigned e = (c >> 2) & 7, m = c & 3;
    const float v = e ? (1.0f + m / 4.0f) * (float)(1 << e) / 8.0f : m / 16.0f;
    return (c & 32) ? -v : v;
}

int main() {
    static v8i ha[64], hb[64];
    static float A[16][128], B[128][16];
    srand(13);
    memset(ha, 0, sizeof ha);
    memset(hb, 0, sizeof hb);
    const unsigned bcodes[3] = {0, 8, 16};
    for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 32; ++j) {
            const unsigned ca = rand() & 31, cb = bcodes[rand() % 3];
            const int bit = 6 * j;
            ha[l][bit / 32] |= (int)(ca << (bit % 32));
            hb[l][bit / 32] |= (int)(cb << (bit % 32));
            if (bit % 32 > 26) {
                ha[l][bit / 32 + 1] |= (int)(ca >> (32 - bit % 32));
                hb[l][bit / 32 + 1] |= (int)(cb >> (32 - bit % 32));
            }
            A[l & 15][32 * (l >> 4) + j] = e2m3(ca);
            B[32 * (l >> 4) + j][l & 15] = (float)cb;  // the code; decoded per format below
        }
    printf("decodings: e2m3 8 -> %g, 16 -> %g; e3m2 8 -> %g, 16 -> %g\n", e2m3(8), e2m3(16), e3m2(8), e3m2(16));
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
    for (int fmt = 2; fmt <= 3; ++fmt) {
        if (fmt == 2)
            hipLaunchKernelGGL((kern<2, 2>), dim3(1), dim3(64), 0, 0, da, db, dc);
        else
            hipLaunchKernelGGL((kern<2, 3>), dim3(1), dim3(64), 0, 0, da, db, dc);
        v4f hc[64];
        hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost);
        for (int l = 0; l < 64; ++l)
            for (int e = 0; e < 4; ++e) {
                const int row = 4 * (l >> 4) + e, col = l & 15;
                double ref = 0;
                for (int k = 0; k < 128; ++k) {
                    const unsigned cb = (unsigned)B[k][col];
                    ref += (double)A[row][k] * (fmt == 2 ? e2m3(cb) : e3m2(cb));
                }
                if ((double)hc[l][e] != ref) {
                    if (bad < 8) printf("mismatch fmt %d row %d col %d: gpu %.5f ref %.5f\n", fmt, row, col, hc[l][e], ref);
                    ++bad;
                }
            }
    }
    printf("fp6 x {fp6, bf6} dual reading: %s (%d mismatches)\n", bad ? "FAIL" : "ok", bad);
    long long cyc[3];
    const int n = 512;
    hipLaunchKernelGGL((rate<2, 4>), dim3(1), dim3(64), 0, 0, da, db, dc, dcyc, n);
    hipMemcpy(&cyc[0], dcyc, sizeof(long long), hipMemcpyDeviceToHost);
    hipLaunchKernelGGL((rate<2, 2>), dim3(1), dim3(64), 0, 0, da, db, dc, dcyc, n);
    hipMemcpy(&cyc[1], dcyc, sizeof(long long), hipMemcpyDeviceToHost);
    hipLaunchKernelGGL((rate<2, 3>), dim3(1), dim3(64), 0, 0, da, db, dc, dcyc, n);
    hipMemcpy(&cyc[2], dcyc, sizeof(long long), hipMemcpyDeviceToHost);
    printf("cycles per MFMA (one wave, 8 accumulators): fp6xfp4 %.2f, fp6xfp6 %.2f, fp6xbf6 %.2f\n",
           (double)cyc[0] / (8.0 * n), (double)cyc[1] / (8.0 * n), (double)cyc[2] / (8.0 * n));
    return bad != 0;
}
