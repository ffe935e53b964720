// Device-side encode of a loaded SiteSet.
//
// Hoists the per-pair `major_minor_symbols` calls of single_weighted_ld_pair
// (lib.rs:400-408 -> lib.rs:126-140) to one pass per site: histogram over all
// n_seqs symbols (lib.rs:98-104, SiteSet keeps it per site, lib.rs:194-196),
// major/minor with the reference's tie rule, then one code byte per
// (site, sequence):  bit0 = symbol is major or minor (the "in" mask of
// lib.rs:435), bit1 = symbol is major (lib.rs:430,432).  Sites whose major or
// minor is None get ok=0 (the pair returns None, lib.rs:400-408) and zero codes.
// Sequences are zero-padded to NP (a multiple of 64) and sites to LP (a
// multiple of 256); padding carries code 0 and weight 0, so it adds nothing.
#include "kernels.hpp"

namespace wld {

__global__ __launch_bounds__(256) void encode_kernel(const uint8_t *__restrict__ sites,
                                                      const uint32_t *__restrict__ site_index, uint32_t L,
                                                      uint32_t N, uint32_t NP, uint8_t *__restrict__ codes,
                                                      uint8_t *__restrict__ site_ok) {
    __shared__ uint32_t h[6];
    const uint32_t s = blockIdx.x;
    const uint32_t tid = threadIdx.x;
    if (tid < 6) h[tid] = 0;
    __syncthreads();
    // site_index (device pre-pass): row s of the filtered set is raw row site_index[s]
    const uint8_t *row = sites + (size_t)(site_index && s < L ? site_index[s] : s) * N;
    if (s < L) {
        uint32_t c[6] = {0, 0, 0, 0, 0, 0};
        for (uint32_t k = tid; k < N; k += 256) {
            uint32_t v = row[k];
            v = v < 6 ? v : 5;
#pragma unroll
            for (int q = 0; q < 6; ++q) c[q] += (v == (uint32_t)q);
        }
#pragma unroll
        for (int q = 0; q < 6; ++q)
            if (c[q]) atomicAdd(&h[q], c[q]);
    }
    __syncthreads();
    // lib.rs:126-140
    int maj = -1, mnr = -1;
    for (int q = 0; q <= 4; ++q) {
        uint32_t cm = maj >= 0 ? h[maj] : 0u, cn = mnr >= 0 ? h[mnr] : 0u;
        if (h[q] > cm) {
            mnr = maj;
            maj = q;
        } else if (h[q] > cn) {
            mnr = q;
        }
    }
    const bool ok = (s < L) && maj >= 0 && mnr >= 0;
    uint8_t *out = codes + (size_t)s * NP;
    for (uint32_t k = tid; k < NP; k += 256) {
        uint8_t code = 0;
        if (ok && k < N) {
            int v = row[k];
            code = (v == maj) ? (kCodeIn | kCodeMaj) : (v == mnr ? kCodeIn : 0);
        }
        out[k] = code;
    }
    if (tid == 0) site_ok[s] = ok ? 1 : 0;
}

// w_pad[k] = k < N ? w[k] : 0, and wstats = {max finite |w|, min nonzero
// finite |w|, any non-finite (1/0)} for the kernel choice (capi.hip).
__global__ __launch_bounds__(256) void weight_prep_kernel(const float *__restrict__ w, uint32_t N, uint32_t NP,
                                                           float *__restrict__ w_pad, float *__restrict__ wstats) {
    __shared__ float smax[256], smin[256], snf[256];
    const uint32_t tid = threadIdx.x;
    float mx = 0.0f, mn = INFINITY, nf = 0.0f;
    for (uint32_t k = tid; k < NP; k += 256) {
        float v = k < N ? w[k] : 0.0f;
        w_pad[k] = v;
        if (k < N) {
            if (!isfinite(v)) {
                nf = 1.0f;
            } else {
                float a = fabsf(v);
                mx = fmaxf(mx, a);
                if (a > 0.0f) mn = fminf(mn, a);
            }
        }
    }
    smax[tid] = mx;
    smin[tid] = mn;
    snf[tid] = nf;
    __syncthreads();
    for (uint32_t st = 128; st > 0; st >>= 1) {
        if (tid < st) {
            smax[tid] = fmaxf(smax[tid], smax[tid + st]);
            smin[tid] = fminf(smin[tid], smin[tid + st]);
            snf[tid] = fmaxf(snf[tid], snf[tid + st]);
        }
        __syncthreads();
    }
    if (tid == 0) {
        wstats[0] = smax[0];
        wstats[1] = smin[0];
        wstats[2] = snf[0];
    }
}

void launch_encode(const uint8_t *d_sites, const uint32_t *site_index, size_t L, size_t N, size_t LP, size_t NP,
                   uint8_t *codes, uint8_t *site_ok, hipStream_t s) {
    hipLaunchKernelGGL(encode_kernel, dim3((unsigned)LP), dim3(256), 0, s, d_sites, site_index, (uint32_t)L,
                       (uint32_t)N, (uint32_t)NP, codes, site_ok);
}

void launch_weight_prep(const float *d_w, size_t N, size_t NP, float *w_pad, float *wstats, hipStream_t s) {
    hipLaunchKernelGGL(weight_prep_kernel, dim3(1), dim3(256), 0, s, d_w, (uint32_t)N, (uint32_t)NP, w_pad, wstats);
}

}  // namespace wld
