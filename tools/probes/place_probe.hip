// Workgroup placement probe: for each block of a 2048-block grid shaped like
// the fp6 screen (256 threads, 34 KB LDS: four per CU), wave 0 records
// HW_ID (wave, SIMD, CU, SH, SE, workgroup slot), XCC_ID and its start and
// end times.  Output: one line per block.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ __launch_bounds__(256) void probe(unsigned *o, unsigned long long *t) {
    __shared__ unsigned pad[34 * 256];
    const unsigned long long t0 = wall_clock64();
    pad[threadIdx.x * 34] = threadIdx.x;
    __syncthreads();
    unsigned hw, x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    // hold the slot ~20 us so one round is resident together
    const unsigned long long s0 = wall_clock64();
    while (wall_clock64() - s0 < 2000) __builtin_amdgcn_s_sleep(8);
    if (threadIdx.x == 0) {
        o[2 * blockIdx.x] = hw;
        o[2 * blockIdx.x + 1] = x + pad[(threadIdx.x + 1) * 34 % (34 * 256)] * 0;
        t[2 * blockIdx.x] = t0;
        t[2 * blockIdx.x + 1] = wall_clock64();
    }
}
int main() {
    const int n = 2048;
    unsigned *o; unsigned long long *t;
    if (hipMalloc(&o, n * 8) || hipMalloc(&t, n * 16)) return 1;
    hipLaunchKernelGGL(probe, dim3(n), dim3(256), 0, 0, o, t);
    if (hipDeviceSynchronize()) return 2;
    std::vector<unsigned> h(2 * n); std::vector<unsigned long long> ht(2 * n);
    hipMemcpy(h.data(), o, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(ht.data(), t, n * 16, hipMemcpyDeviceToHost);
    unsigned long long tmin = ~0ull;
    for (int b = 0; b < n; ++b) tmin = ht[2 * b] < tmin ? ht[2 * b] : tmin;
    for (int b = 0; b < n; ++b) {
        const unsigned w = h[2 * b];
        printf("%d wave=%u simd=%u cu=%u sh=%u se=%u tg=%u xcc=%u t0=%llu t1=%llu\n", b, w & 15, (w >> 4) & 3,
               (w >> 8) & 15, (w >> 12) & 1, (w >> 13) & 7, (w >> 16) & 15, h[2 * b + 1] & 15, ht[2 * b] - tmin,
               ht[2 * b + 1] - tmin);
    }
    return 0;
}
