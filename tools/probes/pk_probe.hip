// Packed-f32 hazard probe: which producer -> consumer pair
// around v_pk_add_f32 / v_pk_mul_f32 reads or leaves a stale value, and in
// which lanes, with and without matrix-pipe load on the same SIMD.
//
// Each 512-thread workgroup holds 8 waves, two per SIMD: waves 0-3 keep the
// matrix pipe busy (v_mfma_i32_16x16x64_i8 chains, like the one-plane pair
// kernel's co-resident waves) when `load` is set; waves 4-7 run a fixed
// instruction sequence in inline asm (explicit VGPRs, so the compiler inserts
// no wait states) with 0..8 wait states between producer and consumer, many
// times, and count per lane the results that differ from the plain-C value.
//   seq 0  v_pk_add_f32 -> v_add_f32 reading both halves        (pk -> VALU RAW)
//   seq 1  v_pk_add_f32 -> v_pk_mul_f32 reading the pair        (pk -> pk RAW)
//   seq 2  v_cvt_f32_f64 (DP) -> v_pk_add_f32 reading it         (DP -> pk RAW)
//   seq 3  v_pk_add_f32 v[44:45], then v_mov_b32 v44 (overwrite) (pk -> VALU WAW)
//   seq 4  v_rcp_f32 (trans) -> v_pk_add_f32 reading it          (trans -> pk RAW)
//   seq 5  v_add_f32 -> v_add_f32 (plain VALU RAW, control)
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/probes/pk_probe.hip -o tools/probes/pk_probe
//   tools/probes/pk_probe        (prints one line per (seq, wait states, load))
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));

template <int SEQ, int W>
__device__ __forceinline__ float run_seq(float x, float y, float z) {
    float r;
    // inputs staged into fixed registers, a settle gap, the probed pair, then
    // the result copied out after a long gap (s_nop 7 x2)
#define PRE                                                                                      \
    "v_mov_b32 v40, %1\n v_mov_b32 v41, %2\n v_mov_b32 v42, %2\n v_mov_b32 v43, %1\n"           \
    "v_cvt_f64_f32 v[48:49], %2\n v_mov_b32 v50, %3\n s_nop 7\n s_nop 7\n"
#define POST "s_nop 7\n s_nop 7\n"
#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50"
    if constexpr (SEQ == 0) {
        if constexpr (W == 0)
            asm volatile(PRE "v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n v_add_f32 v46, v44, v45\n" POST
                         "v_mov_b32 %0, v46" : "=v"(r) : "v"(x), "v"(y), "v"(z) : CLOB);
        else if constexpr (W == 1)
            asm volatile(PRE "v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 0\n v_add_f32 v46, v44, v45\n" POST
                         "v_mov_b32 %0, v46" : "=v"(r) : "v"(x), "v"(y), "v"(z) : CLOB);
        else if constexpr (W == 2)
            asm volatile(PRE "v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 1\n v_add_f32 v46, v44, v45\n" POST
                         "v_mov_b32 %0, v46" : "=v"(r) : "v"(x), "v"(y), "v"(z) : CLOB);
        else
            asm volatile(PRE "v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 3\n v_add_f32 v46, v44, v45\n" POST
                         "v_mov_b32 %0, v46" : "=v"(r) : "v"(x), "v"(y), "v"(z) : CLOB);
    } else if constexpr (SEQ == 1) {
        if constexpr (W == 0)
            asm volatile(PRE "v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n v_pk_mul_f32 v[46:47], v[44:45], v[40:41]\n"
                         POST "v_add_f32 %0, v46, v47" : "=v"(r) : "v"(x), "v"(y), "v"(z) : CLOB);
        else if constexpr (W == 1)
            asm volatile(PRE "v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 0\n v_pk_mul_f32 v[46:47], v[44:45], "
                         "v[40:41]\n" POST "v_add_f32 %0, v46, v47" : "=v"(r) : "v"(x), "v"(y), "v"(z) : CLOB);
        else if constexpr (W == 2)
            asm volatile(PRE "v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 1\n v_pk_mul_f32 v[46:47], v[44:45], "
                         "v[40:41]\n" POST "v_add_f32 %0, v46, v47" : "=v"(r) : "v"(x), "v"(y), "v"(z) : CLOB);
        else
            asm volatile(PRE "v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 3\n v_pk_mul_f32 v[46:47], v[44:45], "
                         "v[40:41]\n" POST "v_add_f32 %0, v46, v47" : "=v"(r) : "v"(x), "v"(y), "v"(z) : CLOB);
    } else if constexpr (SEQ == 2) {
        if constexpr (W == 0)
            asm volatile(PRE "v_cvt_f32_f64 v41, v[48:49]\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n" POST
                         "v_add_f32 %0, v44, v45" : "=v"(r) : "v"(x), "v"(y), "v"(z) : CLOB);
        else if constexpr (W == 1)
            asm volatile(PRE "v_cvt_f32_f64 v41, v[48:49]\n s_nop 0\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n"
                         POST "v_add_f32 %0, v44, v45" : "=v"(r) : "v"(x), "v"(y), "v"(z) : CLOB);
        else if constexpr (W == 2)
            asm volatile(PRE "v_cvt_f32_f64 v41, v[48:49]\n s_nop 1\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n"
                         POST "v_add_f32 %0, v44, v45" : "=v"(r) : "v"(x), "v"(y), "v"(z) : CLOB);
        else
            asm volatile(PRE "v_cvt_f32_f64 v41, v[48:49]\n s_nop 3\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n"
                         POST "v_add_f32 %0, v44, v45" : "=v"(r) : "v"(x), "v"(y), "v"(z) : CLOB);
    } else if constexpr (SEQ == 3) {
        if constexpr (W == 0)
            asm volatile(PRE "v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n v_mov_b32 v44, v50\n" POST
                         "v_mov_b32 %0, v44" : "=v"(r) : "v"(x), "v"(y), "v"(z) : CLOB);
        else if constexpr (W == 1)
            asm volatile(PRE "v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 0\n v_mov_b32 v44, v50\n" POST
                         "v_mov_b32 %0, v44" : "=v"(r) : "v"(x), "v"(y), "v"(z) : CLOB);
        else if constexpr (W == 2)
            asm volatile(PRE "v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 1\n v_mov_b32 v44, v50\n" POST
                         "v_mov_b32 %0, v44" : "=v"(r) : "v"(x), "v"(y), "v"(z) : CLOB);
        else
            asm volatile(PRE "v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 3\n v_mov_b32 v44, v50\n" POST
                         "v_mov_b32 %0, v44" : "=v"(r) : "v"(x), "v"(y), "v"(z) : CLOB);
    } else if constexpr (SEQ == 4) {
        if constexpr (W == 0)
            asm volatile(PRE "v_rcp_f32 v41, v41\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n" POST
                         "v_add_f32 %0, v44, v45" : "=v"(r) : "v"(x), "v"(y), "v"(z) : CLOB);
        else if constexpr (W == 1)
            asm volatile(PRE "v_rcp_f32 v41, v41\n s_nop 0\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n" POST
                         "v_add_f32 %0, v44, v45" : "=v"(r) : "v"(x), "v"(y), "v"(z) : CLOB);
        else if constexpr (W == 2)
            asm volatile(PRE "v_rcp_f32 v41, v41\n s_nop 1\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n" POST
                         "v_add_f32 %0, v44, v45" : "=v"(r) : "v"(x), "v"(y), "v"(z) : CLOB);
        else
            asm volatile(PRE "v_rcp_f32 v41, v41\n s_nop 3\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n" POST
                         "v_add_f32 %0, v44, v45" : "=v"(r) : "v"(x), "v"(y), "v"(z) : CLOB);
    } else {
        if constexpr (W == 0)
            asm volatile(PRE "v_add_f32 v44, v40, v41\n v_add_f32 v46, v44, v43\n" POST "v_mov_b32 %0, v46"
                         : "=v"(r) : "v"(x), "v"(y), "v"(z) : CLOB);
        else
            asm volatile(PRE "v_add_f32 v44, v40, v41\n s_nop 0\n v_add_f32 v46, v44, v43\n" POST "v_mov_b32 %0, v46"
                         : "=v"(r) : "v"(x), "v"(y), "v"(z) : CLOB);
    }
    return r;
}

template <int SEQ>
__device__ __forceinline__ float expect(float x, float y, float z) {
    if constexpr (SEQ == 0) return (x + y) + (y + x);
    if constexpr (SEQ == 1) return (x + y) * x + (y + x) * y;
    if constexpr (SEQ == 2) return (x + y) + (y + x);  // v41 = (float)(double)y = y
    if constexpr (SEQ == 3) return z;
    if constexpr (SEQ == 4) return (x + y) + (__builtin_amdgcn_rcpf(y) + x);
    return (x + y) + x;
}

template <int SEQ, int W>
__global__ __launch_bounds__(512) void probe(const float *in, unsigned *bad, int iters, int load, v4i *sink) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (wave < 4) {
        if (!load) return;
        v4i a = {lane, 3, 5, 7}, b = {1, lane, 2, 9}, c = {0, 0, 0, 0}, d = c, e = c, f = c;
        for (int i = 0; i < iters * 6; ++i) {
            c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
            d = __builtin_amdgcn_mfma_i32_16x16x64_i8(b, a, d, 0, 0, 0);
            e = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, a, e, 0, 0, 0);
            f = __builtin_amdgcn_mfma_i32_16x16x64_i8(b, b, f, 0, 0, 0);
        }
        sink[blockIdx.x * 256 + threadIdx.x] = c + d + e + f;
        return;
    }
    const int t = blockIdx.x * 256 + (threadIdx.x - 256);
    const float x = in[3 * t], y = in[3 * t + 1], z = in[3 * t + 2];
    const float want = expect<SEQ>(x, y, z);
    unsigned nb = 0;
    for (int i = 0; i < iters; ++i) {
        const float got = run_seq<SEQ, W>(x, y, z);
        nb += __float_as_uint(got) != __float_as_uint(want);
    }
    if (nb) atomicAdd(&bad[lane], nb);
}

template <int SEQ, int W>
void one(const float *din, unsigned *dbad, v4i *dsink, int blocks, int iters, int load) {
    hipMemset(dbad, 0, 64 * sizeof(unsigned));
    hipLaunchKernelGGL((probe<SEQ, W>), dim3(blocks), dim3(512), 0, 0, din, dbad, iters, load, dsink);
    std::vector<unsigned> h(64);
    hipMemcpy(h.data(), dbad, 64 * sizeof(unsigned), hipMemcpyDeviceToHost);
    unsigned long long tot = 0, q[4] = {0, 0, 0, 0};
    for (int l = 0; l < 64; ++l) {
        tot += h[l];
        q[l / 16] += h[l];
    }
    printf("seq %d wait_states %d mfma_load %d: bad %llu of %llu (lanes 0-15 %llu, 16-31 %llu, 32-47 %llu, 48-63 %llu)\n",
           SEQ, W == 4 ? 4 : W, load, tot, (unsigned long long)blocks * 256 * iters, q[0], q[1], q[2], q[3]);
}

template <int SEQ>
void seq_all(const float *din, unsigned *dbad, v4i *dsink, int blocks, int iters) {
    for (int load = 0; load < 2; ++load) {
        one<SEQ, 0>(din, dbad, dsink, blocks, iters, load);
        one<SEQ, 1>(din, dbad, dsink, blocks, iters, load);
        if constexpr (SEQ != 5) {
            one<SEQ, 2>(din, dbad, dsink, blocks, iters, load);
            one<SEQ, 4>(din, dbad, dsink, blocks, iters, load);
        }
    }
}

int main() {
    const int blocks = 2048, iters = 400;
    std::vector<float> in(3 * blocks * 256);
    unsigned s = 12345;
    for (auto &v : in) {
        s = s * 1664525u + 1013904223u;
        v = 0.5f + (float)(s >> 8) * 0x1p-24f;
    }
    float *din;
    unsigned *dbad;
    v4i *dsink;
    hipMalloc(&din, in.size() * sizeof(float));
    hipMalloc(&dbad, 64 * sizeof(unsigned));
    hipMalloc(&dsink, (size_t)blocks * 256 * sizeof(v4i));
    hipMemcpy(din, in.data(), in.size() * sizeof(float), hipMemcpyHostToDevice);
    seq_all<0>(din, dbad, dsink, blocks, iters);
    seq_all<1>(din, dbad, dsink, blocks, iters);
    seq_all<2>(din, dbad, dsink, blocks, iters);
    seq_all<3>(din, dbad, dsink, blocks, iters);
    seq_all<4>(din, dbad, dsink, blocks, iters);
    seq_all<5>(din, dbad, dsink, blocks, iters);
    const hipError_t e = hipDeviceSynchronize();
    printf("done: %s\n", hipGetErrorString(e));
    return e == hipSuccess ? 0 : 1;
}
