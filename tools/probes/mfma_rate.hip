// MFMA i8 throughput probe: grid of 256-thread workgroups (2 per CU by launch
// bounds), each wave issuing ITERS x 12 independent v_mfma_i32_32x32x32_i8 on
// register operands.  Prints achieved int8 TOPS; clock from s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ __launch_bounds__(256, 2) void k(int iters, int *out, unsigned long long *clk) {
    v16i acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = v16i{};
    v4i a = {(int)threadIdx.x, 1, 2, 3}, b = {3, (int)threadIdx.x, 5, 7};
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        asm volatile("" : "+v"(a), "+v"(b));
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[i], 0, 0, 0);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    int s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] ^ acc[i][15];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

template <int NACC>
void run(int grid, int iters) {
    int *out; unsigned long long *clk;
    hipMalloc(&out, grid * 256 * 4); hipMalloc(&clk, grid * 8);
    hipLaunchKernelGGL(k<NACC>, dim3(grid), dim3(256), 0, 0, iters, out, clk);
    hipDeviceSynchronize();
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<NACC>, dim3(grid), dim3(256), 0, 0, iters, out, clk);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c; hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost);
    double ops = (double)grid * 4 * iters * NACC * 65536.0;
    printf("nacc=%d grid=%d iters=%d ms=%.3f TOPS=%.0f wave_cycles=%llu cyc/mfma/wave=%.1f ghz_est=%.2f\n", NACC, grid,
           iters, ms, ops / ms / 1e9, c, (double)c / (iters * NACC), (double)c / (ms * 1e6));
}

int main() {
    run<12>(512, 2000);
    run<12>(512, 20000);
    run<12>(1024, 10000);
    run<8>(512, 20000);
    run<4>(512, 20000);
    return 0;
}
