// Probe: where does a global_load_lds_dwordx4 aimed at LDS offsets >= 64 KiB land?
// One workgroup of 64 threads, 80 KiB of static LDS.  Fill LDS with a marker,
// DMA 1 KiB of a pattern to destination offset D (one wave), wait, then dump
// the whole LDS to global memory.  The host reports where the pattern appeared.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef __attribute__((address_space(3))) void lds_void;
constexpr int kLds = 80 * 1024;

__global__ __launch_bounds__(64) void probe(const uint8_t *src, uint32_t dst_off, uint8_t *dump) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLds];
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t * 4; i < kLds; i += 256) *reinterpret_cast<uint32_t *>(lds + i) = 0xEEEEEEEEu;
    __syncthreads();
    __builtin_amdgcn_global_load_lds(src + t * 16, (lds_void *)(lds + dst_off), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (uint32_t i = t * 4; i < kLds; i += 256) *reinterpret_cast<uint32_t *>(dump + i) = *reinterpret_cast<uint32_t *>(lds + i);
}

int main() {
    uint8_t *src, *dump;
    hipMalloc(&src, 1024);
    hipMalloc(&dump, kLds);
    std::vector<uint8_t> h(1024);
    for (int i = 0; i < 1024; ++i) h[i] = (uint8_t)(i * 7 + 1) | 0x01;
    hipMemcpy(src, h.data(), 1024, hipMemcpyHostToDevice);
    const uint32_t offs[] = {0, 32768, 64512, 65536, 66560, 67584, 73728};
    for (uint32_t off : offs) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, src, off, dump);
        std::vector<uint8_t> d(kLds);
        if (hipMemcpy(d.data(), dump, kLds, hipMemcpyDeviceToHost) != hipSuccess) { printf("copy failed\n"); return 1; }
        // find the pattern
        int found = -1;
        for (int p = 0; p + 1024 <= kLds; p += 16)
            if (d[p] == h[0] && d[p + 1] == h[1] && d[p + 1023] == h[1023]) { found = p; break; }
        int changed = 0;
        for (int p = 0; p < kLds; ++p) changed += d[p] != 0xEE;
        printf("dst_off=%u found_at=%d bytes_changed=%d\n", off, found, changed);
    }
    return 0;
}
