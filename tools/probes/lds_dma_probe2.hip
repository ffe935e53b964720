// Probe 2: two or more workgroups per CU, each with 68 KiB of static LDS,
// repeatedly DMA workgroup-specific patterns into the high part of their LDS
// (buffer-1-like offsets 33792..67583) and verify every byte of their own LDS.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef __attribute__((address_space(3))) void lds_void;
constexpr int kLds = 68352;

__global__ __launch_bounds__(256, 2) void probe(const uint32_t *src, uint32_t iters, uint32_t *errors) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLds];
    const uint32_t t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
    uint32_t err = 0;
    for (uint32_t it = 0; it < iters; ++it) {
        const uint32_t tag = (blockIdx.x * 131u + it * 7u) & 0xFFFFu;
        // fill: every dword = (tag << 16) | (dword index & 0xFFFF)
        for (uint32_t i = t; i < kLds / 4; i += 256) reinterpret_cast<uint32_t *>(lds)[i] = (tag << 16) | (i & 0xFFFF);
        __syncthreads();
        // 17 DMAs per wave: 1 KB blocks at offsets 33792 + (17*wave + j)*1024 (clamped to the array)
        for (uint32_t j = 0; j < 8; ++j) {
            const uint32_t blk = 33 + wave * 8 + j;  // 1 KB blocks 33..64 -> offsets 33792..66559
            __builtin_amdgcn_global_load_lds(src + (size_t)(blockIdx.x * 64 + blk) * 256 + lane * 4,
                                             (lds_void *)(lds + blk * 1024), 16, 0, 0);
        }
        if (wave == 0)
            __builtin_amdgcn_global_load_lds(src + (size_t)(blockIdx.x * 64 + 65) * 256 + lane * 4,
                                             (lds_void *)(lds + 65 * 1024), 16, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (uint32_t i = t; i < kLds / 4; i += 256) {
            const uint32_t blk = i / 256;
            uint32_t want = (tag << 16) | (i & 0xFFFF);
            if (blk >= 33 && blk <= 65) want = src[(size_t)(blockIdx.x * 64 + blk) * 256 + (i % 256)];
            err += reinterpret_cast<uint32_t *>(lds)[i] != want;
        }
        __syncthreads();
    }
    if (err) atomicAdd(errors + blockIdx.x % 1024, err);
}

int main(int argc, char **argv) {
    const int nwg = argc > 1 ? atoi(argv[1]) : 1024;
    const uint32_t iters = argc > 2 ? atoi(argv[2]) : 50;
    uint32_t *src, *errors;
    const size_t n = (size_t)(nwg * 64 + 80) * 256;
    hipMalloc(&src, n * 4);
    hipMalloc(&errors, 1024 * 4);
    hipMemset(errors, 0, 1024 * 4);
    std::vector<uint32_t> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = (uint32_t)(i * 2654435761u) ^ 0xA5A5A5A5u;
    hipMemcpy(src, h.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(nwg), dim3(256), 0, 0, src, iters, errors);
    std::vector<uint32_t> e(1024);
    if (hipMemcpy(e.data(), errors, 1024 * 4, hipMemcpyDeviceToHost) != hipSuccess) { printf("failed\n"); return 1; }
    uint64_t tot = 0; int nbad = 0;
    for (auto x : e) { tot += x; nbad += x != 0; }
    printf("nwg=%d iters=%u error_dwords=%llu bad_wg_slots=%d\n", nwg, iters, (unsigned long long)tot, nbad);
    return 0;
}
