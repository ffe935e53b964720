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
constexpr uint32_t kRowLds = 8192;  // site rows up to this many sequences are staged in LDS (per wave)
}  // namespace

// One wavefront per raw site (4 per workgroup): symbol histogram over all N
// (lib.rs:98-104, Unknown included) by per-lane counts and a wave reduction,
// major/minor (lib.rs:126-140), the keep flag of is_site_of_interest, and the
// site's Henikoff table: tab[k] = 1/(distinct * h[k]) for k in ACGT- and
// tab[5] = (sequential f32 sum of the row's ACGT- contributions) / distinct,
// the Unknown fill (lib.rs:360-371).  The fill is summed by one lane in
// sequence order (the reference's order), out of the wave's LDS copy of the
// row when it fits; it is only needed, and only computed, when the kept site
// has Unknown symbols.
__global__ __launch_bounds__(256) void site_stats_kernel(const uint8_t *__restrict__ raw, uint32_t L, uint32_t N,
                                                         uint32_t min_acgt, float min_minor, float max_minor,
                                                         uint8_t *__restrict__ keep, float *__restrict__ tab) {
    __shared__ uint8_t row[4][kRowLds];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t s = blockIdx.x * 4 + wave;
    if (s >= L) return;
    const uint8_t *src = raw + (size_t)s * N;
    const bool stage = N <= kRowLds;
    uint32_t c[6] = {0, 0, 0, 0, 0, 0};
    uint32_t k = lane;
    for (; k + 64 * 7 < N; k += 64 * 8) {  // 8 independent byte loads in flight per lane
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = src[k + 64 * u];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint32_t x = v[u] < 6 ? v[u] : (uint32_t)kSymUnknown;  // SiteSet clamps (lib.rs:53-64)
            if (stage) row[wave][k + 64 * u] = (uint8_t)x;
#pragma unroll
            for (int qq = 0; qq < 6; ++qq) c[qq] += (x == (uint32_t)qq);
        }
    }
    for (; k < N; k += 64) {
        uint32_t x = src[k];
        x = x < 6 ? x : (uint32_t)kSymUnknown;
        if (stage) row[wave][k] = (uint8_t)x;
#pragma unroll
        for (int qq = 0; qq < 6; ++qq) c[qq] += (x == (uint32_t)qq);
    }
    uint32_t h[6];  // wave-uniform after the butterfly reduction
#pragma unroll
    for (int qq = 0; qq < 6; ++qq) {
        uint32_t v = c[qq];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        h[qq] = v;
    }
    int maj = -1, mnr = -1;  // lib.rs:126-140: strict '>' over A,C,G,T,'-'
    for (int qq = 0; qq <= kSymMissing; ++qq) {
        const uint32_t cm = maj >= 0 ? h[maj] : 0u, cn = mnr >= 0 ? h[mnr] : 0u;
        if (h[qq] > cm) {
            mnr = maj;
            maj = qq;
        } else if (h[qq] > cn) {
            mnr = qq;
        }
    }
    const uint32_t acgt = h[0] + h[1] + h[2] + h[3];
    bool ok = false;
    if (acgt > min_acgt && maj >= 0 && mnr >= 0) {
        const float mj = (float)h[maj], mn = (float)h[mnr];
        const float frac = mn / (mn + mj);
        ok = !(frac < min_minor || frac > max_minor);
    }
    uint32_t distinct = 0;
    for (int qq = 0; qq <= kSymMissing; ++qq) distinct += h[qq] > 0;
    const float df = (float)distinct;
    float t[6];
    for (int qq = 0; qq <= kSymMissing; ++qq) t[qq] = 1.0f / (df * (float)h[qq]);
    t[5] = 0.0f;
    if (ok && h[kSymUnknown]) {
        // lane 0 adds in sequence order out of LDS; a row longer than the
        // stage is re-read in stage-sized pieces by the whole wave
        float total = 0.0f;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the staged row's LDS writes
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t j0 = 0; j0 < N; j0 += kRowLds) {
            const uint32_t nj = min(kRowLds, N - j0);
            if (!stage) {
                for (uint32_t j = lane; j < nj; j += 64) row[wave][j] = src[j0 + j];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            if (lane == 0)
                for (uint32_t j = 0; j < nj; ++j) {
                    uint32_t v = row[wave][j];
                    v = v < 6 ? v : (uint32_t)kSymUnknown;
                    if (v <= (uint32_t)kSymMissing) total += t[v];
                }
            __builtin_amdgcn_wave_barrier();
        }
        t[5] = total / df;
    }
    if (lane == 0) {
        keep[s] = ok ? 1 : 0;
        for (int qq = 0; qq < 6; ++qq) tab[(size_t)s * 6 + qq] = t[qq];
    }
}

// Henikoff row sums: w[q] = the sum over kept sites, in site order, of the
// site's table entry for sequence q's symbol (ndarray sum_axis over sites,
// lib.rs:354), one f32 add per site in sequence so the result is the host's
// bit for bit.  The adds of one sequence are a serial chain, and there are only
// N chains (2000 at BASELINE config 4), so the loads feeding them must be
// deep: a 1024-thread workgroup owns 64 sequences; waves 1-15 stream blocks of
// kHkSites kept sites (each site row's 64 code bytes, as dwords when N % 4 ==
// 0, and the site's 6-entry table) into double-buffered LDS while wave 0 runs
// the 64 add chains out of the other buffer.
constexpr uint32_t kHkSites = 512;
constexpr uint32_t kHkThreads = 1024;
constexpr uint32_t kHkLoaders = kHkThreads - 64;
constexpr uint32_t kHkDwordIters = (kHkSites * 16 + kHkLoaders - 1) / kHkLoaders;  // 9
constexpr uint32_t kHkByteIters = 12;                                              // per batch

// The kept sites' tables in kept order (tabK[k] = tab[site_index[k]]), so the
// Henikoff loaders read them without a dependent index load.
__global__ __launch_bounds__(256) void gather_tab_kernel(const float *__restrict__ tab,
                                                         const uint32_t *__restrict__ site_index, uint32_t n_kept,
                                                         float *__restrict__ tabK) {
    const uint32_t e = blockIdx.x * 256 + threadIdx.x;
    if (e < n_kept * 6) tabK[e] = tab[(size_t)site_index[e / 6] * 6 + e % 6];
}

__device__ __forceinline__ uint32_t clamp_code(uint32_t x) { return x < 6 ? x : (uint32_t)kSymUnknown; }

__global__ __launch_bounds__(kHkThreads) void henikoff_seq_kernel(const uint8_t *__restrict__ raw,
                                                                  const uint32_t *__restrict__ site_index,
                                                                  uint32_t n_kept, uint32_t N,
                                                                  const float *__restrict__ tabK,
                                                                  float *__restrict__ w) {
    __shared__ __attribute__((aligned(16))) uint8_t sCode[2][kHkSites][64];
    __shared__ float sTab[2][kHkSites * 6];
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint32_t q0 = blockIdx.x * 64, q = q0 + lane;
    const uint32_t n_blocks = (n_kept + kHkSites - 1) / kHkSites;
    const bool dwords = (N & 3) == 0;
    // threads [lo_tid, kHkThreads) fill buffer `buf` with site block `blk`;
    // each thread's loads are issued together (fixed, predicated trip counts).
    // Sites past n_kept in the last block are left unwritten: never summed.
    auto load = [&](uint32_t blk, uint32_t buf, uint32_t lo_tid) {
        const uint32_t k0 = blk * kHkSites, nk = min(kHkSites, n_kept - k0);
        const uint32_t nthr = kHkThreads - lo_tid, t = tid - lo_tid;
        if (dwords) {  // 16 lanes per site row: 4 sequences' codes per lane
            uint32_t v[kHkDwordIters];
#pragma unroll
            for (uint32_t i = 0; i < kHkDwordIters; ++i) {
                const uint32_t e = t + i * nthr, k = e >> 4, j = (e & 15) * 4;
                v[i] = 0;
                if (e < nk * 16 && q0 + j < N)
                    v[i] = *reinterpret_cast<const uint32_t *>(raw + (size_t)site_index[k0 + k] * N + q0 + j);
            }
#pragma unroll
            for (uint32_t i = 0; i < kHkDwordIters; ++i) {
                const uint32_t e = t + i * nthr, k = e >> 4, j = (e & 15) * 4;
                if (e < nk * 16) {
                    uint32_t c = 0;
#pragma unroll
                    for (int u = 0; u < 4; ++u) c |= clamp_code((v[i] >> (8 * u)) & 0xFF) << (8 * u);
                    *reinterpret_cast<uint32_t *>(&sCode[buf][k][j]) = c;
                }
            }
        } else {
            for (uint32_t e0 = t; e0 < nk * 64; e0 += kHkByteIters * nthr) {
                uint32_t v[kHkByteIters];
#pragma unroll
                for (uint32_t i = 0; i < kHkByteIters; ++i) {
                    const uint32_t e = e0 + i * nthr, k = e >> 6, j = e & 63;
                    v[i] = 0;
                    if (e < nk * 64 && q0 + j < N) v[i] = raw[(size_t)site_index[k0 + k] * N + q0 + j];
                }
#pragma unroll
                for (uint32_t i = 0; i < kHkByteIters; ++i) {
                    const uint32_t e = e0 + i * nthr, k = e >> 6, j = e & 63;
                    if (e < nk * 64) sCode[buf][k][j] = (uint8_t)clamp_code(v[i]);
                }
            }
        }
        for (uint32_t e = t; e < nk * 6; e += nthr) sTab[buf][e] = tabK[(size_t)k0 * 6 + e];
    };
    if (n_blocks) load(0, 0, 0);
    __syncthreads();
    float acc = 0.0f;
    for (uint32_t blk = 0; blk < n_blocks; ++blk) {
        const uint32_t cur = blk & 1;
        if (wave == 0) {
            const uint32_t nk = min(kHkSites, n_kept - blk * kHkSites);
            uint32_t k = 0;
            for (; k + 16 <= nk; k += 16) {  // LDS reads issued ahead, adds in site order
                float t[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) t[u] = sTab[cur][(k + u) * 6 + sCode[cur][k + u][lane]];
#pragma unroll
                for (int u = 0; u < 16; ++u) acc = acc + t[u];
            }
            for (; k < nk; ++k) acc = acc + sTab[cur][k * 6 + sCode[cur][k][lane]];
        } else if (blk + 1 < n_blocks) {
            load(blk + 1, cur ^ 1, 64);
        }
        __syncthreads();
    }
    if (wave == 0 && q < N) w[q] = acc;
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
    hipLaunchKernelGGL(site_stats_kernel, dim3((unsigned)((L + 3) / 4)), dim3(256), 0, s, raw, (uint32_t)L,
                       (uint32_t)N, min_acgt, min_minor, max_minor, keep, tab);
}

void launch_henikoff(const uint8_t *raw, const uint32_t *site_index, size_t n_kept, size_t N, const float *tab,
                     float *tabK, float *w, hipStream_t s) {
    if (!N) return;
    if (n_kept)
        hipLaunchKernelGGL(gather_tab_kernel, dim3((unsigned)((n_kept * 6 + 255) / 256)), dim3(256), 0, s, tab,
                           site_index, (uint32_t)n_kept, tabK);
    hipLaunchKernelGGL(henikoff_seq_kernel, dim3((unsigned)((N + 63) / 64)), dim3(kHkThreads), 0, s, raw, site_index,
                       (uint32_t)n_kept, (uint32_t)N, tabK, w);
    hipLaunchKernelGGL(normalize_weights_kernel, dim3(1), dim3(1024), 0, s, w, (uint32_t)N);
}

void launch_fill_ones(float *w, size_t N, hipStream_t s) {
    if (!N) return;
    hipLaunchKernelGGL(fill_ones_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, w, (uint32_t)N);
}

}  // namespace wld
