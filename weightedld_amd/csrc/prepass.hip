// Device pre-pass: the site filter and Henikoff
// weights computed on the GPU from the raw SiteSet buffer, bit-for-bit equal to
// the host restatement in host.cpp (and so to lib.rs):
//   is_site_of_interest      lib.rs:309-338 (main.rs:139-143)
//   henikoff_weights         lib.rs:340-380 (main.rs:150-156, on the filtered set)
// The kept-site map is the filter_by site_map (lib.rs:230-251); encode_kernel
// then reads the kept rows of the raw buffer through it (no filtered copy).
#include "kernels.hpp"

namespace wld {

namespace {
constexpr int kSymMissing = 4;  // '-'
constexpr int kSymUnknown = 5;
constexpr uint32_t kRowLds = 32768;  // site rows up to this many sequences are staged in LDS
}  // namespace

// One workgroup per raw site: symbol histogram over all N (lib.rs:98-104,
// Unknown included), major/minor (lib.rs:126-140), the keep flag of
// is_site_of_interest, and the site's Henikoff table: tab[k] = 1/(distinct *
// h[k]) for k in ACGT- and tab[5] = (sequential f32 sum of the row's ACGT-
// contributions) / distinct, the Unknown fill (lib.rs:360-371).  The fill is
// summed by one thread in sequence order (the reference's order); it is only
// needed, and only computed, when the site has Unknown symbols.
__global__ __launch_bounds__(256) void site_stats_kernel(const uint8_t *__restrict__ raw, uint32_t N,
                                                         uint32_t min_acgt, float min_minor, float max_minor,
                                                         uint8_t *__restrict__ keep, float *__restrict__ tab) {
    __shared__ uint32_t h[6];
    __shared__ uint8_t row[kRowLds];
    const uint32_t s = blockIdx.x, tid = threadIdx.x;
    if (tid < 6) h[tid] = 0;
    __syncthreads();
    const uint8_t *src = raw + (size_t)s * N;
    const bool stage = N <= kRowLds;
    uint32_t c[6] = {0, 0, 0, 0, 0, 0};
    for (uint32_t k = tid; k < N; k += 256) {
        uint32_t v = src[k];
        v = v < 6 ? v : kSymUnknown;  // SiteSet clamps codes > Unknown (host.cpp, lib.rs:53-64)
        if (stage) row[k] = (uint8_t)v;
#pragma unroll
        for (int q = 0; q < 6; ++q) c[q] += (v == (uint32_t)q);
    }
#pragma unroll
    for (int q = 0; q < 6; ++q)
        if (c[q]) atomicAdd(&h[q], c[q]);
    __syncthreads();
    if (tid != 0) return;
    int maj = -1, mnr = -1;  // lib.rs:126-140: strict '>' over A,C,G,T,'-'
    for (int q = 0; q <= kSymMissing; ++q) {
        const uint32_t cm = maj >= 0 ? h[maj] : 0u, cn = mnr >= 0 ? h[mnr] : 0u;
        if (h[q] > cm) {
            mnr = maj;
            maj = q;
        } else if (h[q] > cn) {
            mnr = q;
        }
    }
    const uint32_t acgt = h[0] + h[1] + h[2] + h[3];
    bool ok = false;
    if (acgt > min_acgt && maj >= 0 && mnr >= 0) {
        const float mj = (float)h[maj], mn = (float)h[mnr];
        const float frac = mn / (mn + mj);
        ok = !(frac < min_minor || frac > max_minor);
    }
    keep[s] = ok ? 1 : 0;
    uint32_t distinct = 0;
    for (int q = 0; q <= kSymMissing; ++q) distinct += h[q] > 0;
    const float df = (float)distinct;
    float t[6];
    for (int q = 0; q <= kSymMissing; ++q) t[q] = 1.0f / (df * (float)h[q]);
    t[5] = 0.0f;
    if (ok && h[kSymUnknown]) {
        float total = 0.0f;
        for (uint32_t k = 0; k < N; ++k) {
            uint32_t v;
            if (stage) {
                v = row[k];
            } else {
                v = src[k];
                v = v < 6 ? v : kSymUnknown;
            }
            if (v <= (uint32_t)kSymMissing) total += t[v];
        }
        t[5] = total / df;
    }
    for (int q = 0; q < 6; ++q) tab[(size_t)s * 6 + q] = t[q];
}

// One thread per sequence: the sum over kept sites, in site order, of the
// site's table entry for the sequence's symbol (ndarray sum_axis over sites,
// lib.rs:354).
__global__ __launch_bounds__(256) void henikoff_seq_kernel(const uint8_t *__restrict__ raw,
                                                           const uint32_t *__restrict__ site_index, uint32_t n_kept,
                                                           uint32_t N, const float *__restrict__ tab,
                                                           float *__restrict__ w) {
    const uint32_t q = blockIdx.x * 256 + threadIdx.x;
    if (q >= N) return;
    float acc = 0.0f;
    uint32_t k = 0;
    for (; k + 8 <= n_kept; k += 8) {  // loads issued ahead, adds in site order
        uint32_t v[8];
        size_t si[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            si[u] = site_index[k + u];
            v[u] = raw[si[u] * N + q];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc = acc + tab[si[u] * 6 + (v[u] < 6 ? v[u] : (uint32_t)kSymUnknown)];
    }
    for (; k < n_kept; ++k) {
        const size_t si = site_index[k];
        const uint32_t v = raw[si * N + q];
        acc = acc + tab[si * 6 + (v < 6 ? v : (uint32_t)kSymUnknown)];
    }
    w[q] = acc;
}

// w /= max(0, w...) folded with fmax (lib.rs:355; f32::max ignores NaN)
__global__ __launch_bounds__(1024) void normalize_weights_kernel(float *__restrict__ w, uint32_t N) {
    __shared__ float sm[1024];
    float m = 0.0f;
    for (uint32_t q = threadIdx.x; q < N; q += 1024) m = fmaxf(m, w[q]);
    sm[threadIdx.x] = m;
    __syncthreads();
    for (uint32_t o = 512; o > 0; o >>= 1) {
        if (threadIdx.x < o) sm[threadIdx.x] = fmaxf(sm[threadIdx.x], sm[threadIdx.x + o]);
        __syncthreads();
    }
    const float mx = sm[0];
    for (uint32_t q = threadIdx.x; q < N; q += 1024) w[q] = w[q] / mx;
}

__global__ __launch_bounds__(256) void fill_ones_kernel(float *__restrict__ w, uint32_t N) {
    const uint32_t q = blockIdx.x * 256 + threadIdx.x;
    if (q < N) w[q] = 1.0f;
}

void launch_site_stats(const uint8_t *raw, size_t L, size_t N, uint32_t min_acgt, float min_minor, float max_minor,
                       uint8_t *keep, float *tab, hipStream_t s) {
    if (!L) return;
    hipLaunchKernelGGL(site_stats_kernel, dim3((unsigned)L), dim3(256), 0, s, raw, (uint32_t)N, min_acgt, min_minor,
                       max_minor, keep, tab);
}

void launch_henikoff(const uint8_t *raw, const uint32_t *site_index, size_t n_kept, size_t N, const float *tab,
                     float *w, hipStream_t s) {
    if (!N) return;
    hipLaunchKernelGGL(henikoff_seq_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, raw, site_index,
                       (uint32_t)n_kept, (uint32_t)N, tab, w);
    hipLaunchKernelGGL(normalize_weights_kernel, dim3(1), dim3(1024), 0, s, w, (uint32_t)N);
}

void launch_fill_ones(float *w, size_t N, hipStream_t s) {
    if (!N) return;
    hipLaunchKernelGGL(fill_ones_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, w, (uint32_t)N);
}

}  // namespace wld
