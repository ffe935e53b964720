// C ABI of the device hot path (include/weightedld.h).
//
// wld_all_weighted_ld_pairs is the drop-in for all_weighted_ld_pairs
// (lib.rs:578-684).  It is built from the staged calls:
//   wld_load  : H2D of SiteSet.buffer + weights, encode on device
//   wld_run   : pair kernel over the shard's tiles -> staging + segment counts,
//               chunk scan, reference-order gather (order.hip)
//   wld_rows_copy : D2H of the ordered rows
// There is no CPU compute path: without a gfx950 device every device entry
// point fails with WLD_E_NODEV.
#include <algorithm>
#include <cmath>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "common.hpp"
#include "tile_order.hpp"
#include "kernels.hpp"

using namespace wld;

#define HIP_TRY(expr)                                                                               \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess)                                                                       \
            return fail(e_ == hipErrorOutOfMemory ? WLD_E_OOM : WLD_E_HIP, "%s failed: %s (%s:%d)", \
                        #expr, hipGetErrorString(e_), __FILE__, __LINE__);                          \
    } while (0)

#define WLD_TRY(expr)          \
    do {                       \
        int st_ = (expr);      \
        if (st_ != WLD_OK)     \
            return st_;        \
    } while (0)

namespace {

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
};

int ensure(DevBuf &b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.p && b.bytes >= bytes) return WLD_OK;
    if (b.p) {
        (void)hipFree(b.p);
        b.p = nullptr;
        b.bytes = 0;
    }
    hipError_t e = hipMalloc(&b.p, bytes);
    if (e != hipSuccess) {
        b.p = nullptr;
        (void)hipGetLastError();
        return fail(WLD_E_OOM, "hipMalloc(%zu bytes) failed: %s", bytes, hipGetErrorString(e));
    }
    b.bytes = bytes;
    return WLD_OK;
}

void release(DevBuf &b) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
}

template <class T>
T *ptr(DevBuf &b) {
    return reinterpret_cast<T *>(b.p);
}

size_t round_up(size_t x, size_t m) { return (x + m - 1) / m * m; }

}  // namespace

// A run between wld_run_chunks_async (or run_chunks' first phase) and its
// completion: what run_complete needs to check, re-run and assemble it.
struct RunPending {
    bool active = false;
    float thr = 0.f;
    uint32_t lin_begin = 0, lin_end = 0;
    uint64_t pairs = 0;
    unsigned long long *count_out = nullptr;
};

struct wld_ctx {
    int device = 0;
    // a device group (wld_create_multi): one member context per device; the
    // group itself owns no stream or buffers
    std::vector<wld_ctx *> members;
    hipStream_t stream = nullptr;      // where the context's work goes (own_stream or the caller's)
    hipStream_t own_stream = nullptr;  // created with the context
    hipEvent_t ev[7] = {};  // 2..3 pair phase (6: after the screen), 3..4/5 order phase
    RunPending pend;                      // the run between run_enqueue and run_complete
    bool run_dirty = true;                // run state (cursor, chunk totals) may be nonzero: re-initialise
    // mapped pinned {cursor, rows, candidate tiles, sub-blocks} (the scan), then
    // the kernels' guard word (OrderArgs::guard; 0 unless an index was refused)
    unsigned long long *h_cnt = nullptr;
    unsigned long long *d_hcnt = nullptr;
    int cand_set = 0;  // the candidate set (counter words) of the next pass; flips after each scan
    int kernel_pref = WLD_KERNEL_AUTO;
    // wld_set_option (include/weightedld.h)
    bool opt_prefilter = true, opt_tile_rows = false, opt_all_planes = false;
    int opt_screen = 1;  // WLD_OPT_SCREEN: 0 never, 1 auto (default), 2 always, 3 two-plane, 4 exact candidate pairs
    // auto: the largest threshold at which the screen left > half the tiles,
    // and at which the two-plane screen left > a fifth
    float screen_bad_thr = -1.0f;
    // auto: the largest threshold at which the fp6 screen left more than a
    // sixteenth of the tiles (there and below, the i8 screen's tighter bound)
    float fp6_bad_thr = -1.0f;
    // auto: the smallest threshold at which the fp6 screen's sample run found
    // few enough candidate tiles (there and above no sample run is needed)
    float fp6_good_thr = INFINITY;
    DevBuf fp6_probe_buf;  // the sample run's two counts
    float screen2_bad_thr = -1.0f;
    // auto, lib.rs's order: the largest threshold at which the exact candidate
    // pairs were more than a tenth of all pairs (then the full f32 kernel)
    float ref_pairs_bad_thr = -1.0f;
    bool ref_pairs_pass = false;  // the pass staged exact candidate pairs (ref_rows_kernel)
    bool opt_site_major = false, opt_valu_plain = false;
    bool opt_fused_scan = true;  // WLD_OPT_FUSED_SCAN: the chunk scan in the candidate launch's last workgroup
    int opt_test_guard = 0;      // WLD_OPT_TEST_GUARD (tests: a bucket count corrupted before the candidate launch)
    // WLD_OPT_FP6_PAIRS_MIN_TILES: the fp6 screen runs on tile pairs from this
    // many tiles in the run's list, below it one tile per workgroup.  Alone
    // (one pass at a time) single tiles screen rank 0's 1/8 and 1/4 shards of
    // C4 5-7% faster (profiles/r05q, r05s), but in the N>1 step path, where
    // the passes of three contexts overlap, the 1/4 shard steps 6% faster on
    // pairs and the 1/8 shard is even within noise (profiles/r05x); C5 pairs
    // 4.8% faster (profiles/r05j)
    int64_t opt_fp6_pairs_min = 0;  // (tile pairs at every list size: profiles/r05ar/)
    bool opt_i8_pairs = true;    // WLD_OPT_I8_PAIRS: the i8 screen on tile pairs (pre-multiplied images)
    int opt_fp6 = 1;             // WLD_OPT_SCREEN_FP6: 0 off, 1 auto, 2 whenever it applies, 3 auto without the sample run
    bool opt_ref_sums = true;  // WLD_OPT_REF_SUMS: lib.rs's own f32 summation order (default)
    uint64_t opt_staging_rows = 1ull << 25, opt_host_batch_pairs = 1ull << 31;

    // loaded SiteSet
    bool loaded = false;
    size_t L = 0, N = 0, LP = 0, NP = 0;
    DevBuf raw, wraw, codes, w_pad, wstats, site_ok, site_map, planes, frag;
    DevBuf rcodes, rw;       // WLD_OPT_REF_SUMS: codes and weights in lane-class order (ref_layout_kernel)
    // the fp6 screen (fp6_prepare): weight codes, packed operands, constants
    DevBuf w6, f6a, f6b;
    Fp6Screen f6{};
    // the i8 one-plane screen's pre-multiplied images (i8img_prepare, at the
    // first pass that screens on i8 with them)
    DevBuf i8a, i8b;
    I8Screen i8s{};
    bool i8img_ok = false;
    bool fp6_tried = false;   // fp6_prepare ran for this load
    bool fp6_sampled = false; // this pass's screen was chosen by a sample run (fp6_sample)
    bool fp6_ok = false;      // operands built for this load (the weights allow it)
    bool fp6_pass = false;    // the last pass screened on fp6
    bool fp6_better = false;  // ... and its residual is within twice the i8 top digit's (auto)
    double fp6_rel = 0.0, i8_rel = 0.0;  // the two screens' residuals relative to their sums
    bool have_ref = false;   // rcodes/rw hold this load's layout
    uint32_t ref_cls = 0;    // its positions per lane class
    size_t NPr = 0;          // its positions per site
    DevBuf keep, htab, htab_kept, site_index;  // device pre-pass (prepass.hip)
    std::vector<uint64_t> kept_map;  // parent indices of the kept sites (wld_site_map_copy)
    bool prepass_loaded = false;
    bool has_map = false;
    bool use_frag = false;
    int kernel = WLD_KERNEL_VALU;
    bool safe = false;
    int shift = 0;
    int fixed_planes = 3;      // digit planes of the fixed-point weights (3: 23 bits, 4: 31 bits)
    unsigned plane_mask = 7;   // weight-digit planes with a nonzero digit (MFMA)
    MfmaWeightStats wst{7, 1, {0, 0, 0}, {0, 0, 0, 0}};  // digit-plane statistics of the load (MFMA)

    // run state
    DevBuf tiles, cand, seg_cnt, seg_off, chunk_total, chunk_base, counters;
    DevBuf f6_pairs;          // the fp6 screen's tile-pair list of the tile list (pair_fp6_screen2w_kernel)
    uint32_t f6_n_pairs = 0;
    std::vector<uint64_t> chunk_pairs_pre;  // prefix sums of the loaded set's per-chunk pair counts (linear order)
    DevBuf st_a, st_b, st_d, st_dp, st_r2;
    DevBuf out_a, out_b, out_d, out_dp, out_r2;
    uint64_t st_capacity = 0;
    uint32_t tiles_lb = ~0u, tiles_le = ~0u;  // linear chunk range the tile list covers
    uint32_t n_tiles = 0;
    bool have_rows = false;
    bool screened = false;  // the last pass ran a screen
    bool screened2 = false; // ... on two digit planes
    uint64_t rows = 0;
    // the gather goes into the stream behind the scan, before the host has
    // seen the row count, when the previous run had rows:
    // no host round trip between scan and gather; gather_cap: the output
    // rows the enqueued gather may write (0: none enqueued)
    bool spec_gather = false;
    int ev_end = 4;            // the event that ends a pass's scan: 4, or 3 when the scan ran inside the pair launch
    uint64_t gather_cap = 0;
    wld_run_stats stats{};
    // the last pass's phase times, read from its events only when the stats
    // are asked for (materialize_times; ~3 hipEventElapsedTime calls the N>1
    // step loop, which never reads them, does not pay)
    bool times_pending = false;
    bool times_screened = false;
    int times_order_end = 4;
    // per-chunk progress (wld_run_host with a callback): the run's chunk
    // countdowns and log slot counter on the device, the log in mapped pinned
    // host memory (one u64 pair count per completed chunk, ~0 until written)
    DevBuf chunk_left, prog_n;
    unsigned long long *h_plog = nullptr, *d_plog = nullptr;
    size_t plog_cap = 0;
    const std::function<void(uint64_t)> *on_chunk = nullptr;  // set by run_host_range for its runs
    bool prog_pass = false;  // the pass in flight logs its chunks

    ~wld_ctx() {
        for (wld_ctx *m : members) delete m;
        if (!members.empty()) return;
        (void)hipSetDevice(device);
        // work queued on a borrowed stream (wld_set_stream) may still use the
        // buffers: it completes before they are freed
        if (stream && stream != own_stream) (void)hipStreamSynchronize(stream);
        DevBuf *all[] = {&keep, &htab, &htab_kept, &site_index, &raw, &wraw, &codes, &w_pad, &wstats, &site_ok, &site_map, &planes, &frag, &rcodes, &rw, &w6, &f6a, &f6b, &i8a, &i8b, &tiles, &cand, &f6_pairs, &fp6_probe_buf,
                         &seg_cnt, &seg_off, &chunk_total, &chunk_base, &counters, &chunk_left, &prog_n, &st_a, &st_b, &st_d,
                         &st_dp, &st_r2, &out_a, &out_b, &out_d, &out_dp, &out_r2};
        for (DevBuf *b : all) release(*b);
        for (auto &e : ev)
            if (e) (void)hipEventDestroy(e);
        if (h_cnt) (void)hipHostFree(h_cnt);
        if (h_plog) (void)hipHostFree(h_plog);
        if (own_stream) (void)hipStreamDestroy(own_stream);
    }
};

namespace {

// Every single-device entry point starts here; a device group (wld_create_multi)
// supports only wld_load, wld_run_host, wld_all_weighted_ld_pairs and the
// option/kernel/stats calls, which dispatch to its members.
int set_dev(wld_ctx *c) {
    if (!c) return fail(WLD_E_ARG, "null context");
    if (!c->members.empty())
        return fail(WLD_E_STATE, "this call needs a single-device context; a multi-device context supports "
                                 "wld_load, wld_run_host and wld_all_weighted_ld_pairs");
    HIP_TRY(hipSetDevice(c->device));
    return WLD_OK;
}

float event_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0.0f;
    if (a == b) return 0.0f;  // (a phase that ended where it began: no API call)
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) {
        (void)hipGetLastError();
        return -1.0f;
    }
    return ms;
}

// the last completed pass's phase times from its events (run_complete defers them)
void materialize_times(wld_ctx *c) {
    if (!c->times_pending) return;
    c->times_pending = false;
    c->stats.pair_kernel_ms = event_ms(c->ev[2], c->ev[3]);
    c->stats.order_ms = event_ms(c->ev[3], c->ev[c->times_order_end]);
    c->stats.screen_ms = c->times_screened ? event_ms(c->ev[2], c->ev[6]) : 0.0;
}

// fixed-point exponent for the MFMA weight planes: max|w| * 2^shift must fit
// `planes` balanced base-256 digits (|q| <= 127 * (1 + 2^8 + 2^16 [+ 2^24])).
int weight_shift(float maxabs, int planes) {
    const double lim = 127.0 * (1.0 + 256.0 + 65536.0 + (planes == 4 ? 16777216.0 : 0.0));
    int e = 0;
    std::frexp((double)maxabs, &e);  // maxabs = m * 2^e, m in [0.5, 1)
    int shift = (planes == 4 ? 30 : 22) - e;  // maxabs * 2^shift < 2^22 (2^30) < lim
    while (std::ldexp((double)maxabs, shift + 1) <= lim) ++shift;
    while (std::ldexp((double)maxabs, shift) > lim) --shift;
    return shift;
}

double ref_extra_residual(const wld_ctx *c);

// e2m3 (fp6) encoding of a value in [0, 7.5] rounded to the nearest grid
// point, ties to the even code: sign 0, exponent bias 1, 3 mantissa bits.
// The grid steps by 1/8 below 2, by 1/4 in [2, 4) and by 1/2 from 4; within
// each the code's parity is the grid index's, so round-half-even on the index
// (nearbyint) is ties-to-even on the code (an index rounding up to the next
// binade's first point lands on its even code, m = 0).
uint32_t fp6_code(double x, double *rounded) {
    x = std::min(std::max(x, 0.0), 7.5);
    const double step = x < 2.0 ? 0.125 : x < 4.0 ? 0.25 : 0.5;
    const double v = std::min(std::nearbyint(x / step) * step, 7.5);
    *rounded = v;
    if (v < 1.0) return (uint32_t)(v * 8.0);                             // e = 0 (subnormal), m = 8v
    if (v < 2.0) return 8u + (uint32_t)((v - 1.0) * 8.0);                // e = 1
    if (v < 4.0) return 16u + (uint32_t)((v * 0.5 - 1.0) * 8.0);         // e = 2
    return 24u + (uint32_t)((v * 0.25 - 1.0) * 8.0);                     // e = 3
}

// The fp6 screen's operands for this load (pair_mfma.hip): nonnegative
// finite weights, NP <= 16384 (its f32 test on doubled sums), the i8 kernel's
// fragment layout in use.  The weights are rounded to e2m3 at the common
// scale S (of 51 candidates in [3.75, 7.5] / max w) that minimises the L1
// rounding residual; R (in fp6 units) bounds each pass's 2x2-cell L1 distance
// between the screen's sums and the sums the candidate launch computes: the
// rounding, plus the fixed point's 0.5 per sequence (exact mode) and lib.rs's
// f32 summation (9 gamma_m sum w, ref_extra_residual) — both added, so one
// R serves either mode.
// Built at load unless WLD_OPT_SCREEN_FP6 is 0, else on the first run that
// may screen on fp6 after the option is set.
int fp6_prepare(wld_ctx *c) {
    c->fp6_ok = c->fp6_better = false;
    c->fp6_tried = true;
    if (c->kernel != WLD_KERNEL_MFMA || !c->use_frag || !c->wst.nonneg || c->NP > 16384 || c->N == 0) return WLD_OK;
    std::vector<float> w(c->NP);
    HIP_TRY(hipMemcpyAsync(w.data(), c->w_pad.p, c->NP * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    double wmax = 0.0, wsum = 0.0;
    for (size_t k = 0; k < c->N; ++k) wmax = std::max(wmax, (double)w[k]), wsum += (double)w[k];
    if (!(wmax > 0.0) || !std::isfinite(wsum)) return WLD_OK;
    double best_r = INFINITY, best_s = 0.0;
    for (int f = 0; f <= 50; ++f) {
        const double S = 7.5 * (0.5 + 0.01 * f) / wmax;
        double r = 0.0, v;
        for (size_t k = 0; k < c->N; ++k) {
            fp6_code(S * w[k], &v);
            r += std::fabs(S * w[k] - v);
        }
        if (r / S < best_r) best_r = r / S, best_s = S;
    }
    const double S = best_s;
    std::vector<uint8_t> codes(c->NP, 0);
    double r6 = 0.0, sum6 = 0.0, v;
    for (size_t k = 0; k < c->N; ++k) {
        codes[k] = (uint8_t)fp6_code(S * w[k], &v);
        r6 += std::fabs(S * w[k] - v);
        sum6 += v;
    }
    const double u = 0x1p-24, m = (double)(c->N / 8) + 16.0, gamma = m * u / (1.0 - m * u);
    const double extra = S * (9.0 * gamma * wsum + 0.5 * (double)c->N * std::ldexp(1.0, -c->shift) * (1.0 + 9.0 * gamma));
    c->f6.R = (r6 + extra) * (1.0 + 1e-9) + 1e-9 * sum6;
    c->f6.Tg = (float)(2.0 * sum6);  // exact: a multiple of 1/8 below 2^21
    c->f6.NK = (uint32_t)((c->NP + 127) / 128);
    c->fp6_rel = c->f6.R / std::max(sum6, 1e-300);
    // the i8 top digit's: its residual (and the reference's rounding) against
    // the top plane's digit sum, in the same fixed-point units
    uint32_t top = 0;
    for (uint32_t p = 0; p < 4; ++p)
        if (c->wst.plane_mask >> p & 1) top = p;
    const double r8 = (top > 0 ? (double)c->wst.resid[top - 1] : 0.0) + ref_extra_residual(c);
    c->i8_rel = r8 / std::max(std::ldexp((double)c->wst.dsum[top], 8 * (int)top), 1e-300);
    WLD_TRY(ensure(c->w6, c->NP));
    WLD_TRY(ensure(c->f6a, fp6_a_bytes(c->LP, c->NP)));
    WLD_TRY(ensure(c->f6b, fp6_b_bytes(c->LP, c->NP)));
    HIP_TRY(hipMemcpyAsync(c->w6.p, codes.data(), c->NP, hipMemcpyHostToDevice, c->stream));
    launch_frag6(ptr<uint8_t>(c->codes), ptr<uint8_t>(c->w6), c->LP, c->NP, ptr<uint8_t>(c->f6a), ptr<uint8_t>(c->f6b),
                 c->stream);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->f6.a6 = ptr<uint8_t>(c->f6a);
    c->f6.b6 = ptr<uint8_t>(c->f6b);
    c->fp6_ok = true;
    c->fp6_better = c->fp6_rel <= std::max(2.0 * c->i8_rel, 0.02);
    return WLD_OK;
}

// The i8 screen's pre-multiplied operand images of this load (pair_mfma.hip
// pair_i8_screen2w_kernel): the top nonzero digit plane times the site
// indicators, and the codes, 3 bytes per site and sequence; built on the
// context's stream at the first pass that screens on i8 with them.
int i8img_prepare(wld_ctx *c) {
    uint32_t top = 0;
    for (uint32_t p = 0; p < 4; ++p)
        if (c->plane_mask >> p & 1) top = p;
    WLD_TRY(ensure(c->i8a, i8_a_bytes(c->LP, c->NP)));
    WLD_TRY(ensure(c->i8b, i8_b_bytes(c->LP, c->NP)));
    launch_i8img(ptr<uint8_t>(c->codes), ptr<int8_t>(c->planes) + (size_t)top * c->NP, c->LP, c->NP,
                 ptr<uint8_t>(c->i8a), ptr<uint8_t>(c->i8b), c->stream);
    HIP_TRY(hipGetLastError());
    c->i8s = I8Screen{ptr<uint8_t>(c->i8a), ptr<uint8_t>(c->i8b), top};
    c->i8img_ok = true;
    return WLD_OK;
}

int build_tiles(wld_ctx *c, uint32_t lb, uint32_t le);
int ensure_ref_layout(wld_ctx *c);
uint32_t chunks_of(size_t L);
uint32_t chunk_rows_of(size_t L);
void chunk_of_linear_host(uint32_t n, uint32_t i, uint32_t &row, uint32_t &col);
uint64_t pairs_in_chunk(size_t L, uint32_t row, uint32_t col);

int common_load(wld_ctx *c, const uint8_t *d_sites, const float *d_w, const uint64_t *site_map,
                const uint32_t *d_site_index = nullptr) {
    const size_t L = c->L, N = c->N;
    // a new data set: the auto screen policy (thresholds learned on the last
    // one) starts over; the reference-order layout is rebuilt when needed
    c->screen_bad_thr = c->screen2_bad_thr = c->ref_pairs_bad_thr = c->fp6_bad_thr = -1.0f;
    c->fp6_good_thr = INFINITY;
    c->have_ref = false;
    c->LP = round_up(std::max<size_t>(L, 1), kChunk);
    c->NP = round_up(std::max<size_t>(N, 1), kSeqPad);
    WLD_TRY(ensure(c->codes, c->LP * c->NP));
    WLD_TRY(ensure(c->site_ok, c->LP));
    WLD_TRY(ensure(c->w_pad, c->NP * sizeof(float)));
    WLD_TRY(ensure(c->wstats, 4 * sizeof(float)));
    HIP_TRY(hipEventRecord(c->ev[0], c->stream));
    launch_encode(d_sites, d_site_index, L, N, c->LP, c->NP, ptr<uint8_t>(c->codes), ptr<uint8_t>(c->site_ok),
                  c->stream);
    HIP_TRY(hipGetLastError());
    launch_weight_prep(d_w, N, c->NP, ptr<float>(c->w_pad), ptr<float>(c->wstats), c->stream);
    HIP_TRY(hipGetLastError());
    float ws[3] = {0, 0, 0};
    HIP_TRY(hipMemcpyAsync(ws, c->wstats.p, 3 * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));

    const bool finite = ws[2] == 0.0f;
    const float maxabs = ws[0], minabs = ws[1];
    // MFMA planes hold w * 2^shift in fixed point: 3 digit planes (q < 2^23) or
    // 4 (q < 2^31).  Each weight is then within 0.5 / q_min relative of its f32
    // value; AUTO requires that to be <= 2^-19 (sums of nonnegative weights,
    // any cell of the 2x2 table included, keep that relative error, so d and
    // r2 move by ~1e-6 at most: DESIGN.md §5), i.e. min|w| >= 2^-4 max|w| for
    // 3 planes and >= 2^-12 max|w| for 4; wider ranges take the f32 kernel.
    // The int32 accumulators hold X = S(minor) + 2 S(major) and Y = S(minor)
    // with |X| + |Y| <= 3 * 128 * NP (pair_mfma.hip, Acc16::get): NP < 2^31 / 384;
    // 4 planes fold two planes into int32 (NP <= 65024).
    constexpr size_t kMfmaMaxNP = 5592320, kMfma4MaxNP = 65024;
    const bool mfma_fits = c->NP <= kMfmaMaxNP;
    const bool range3 = minabs >= maxabs * 0x1p-4f, range4 = minabs >= maxabs * 0x1p-12f;
    const bool mfma_ok = mfma_supported() && mfma_fits && finite && maxabs > 0.0f &&
                         (range3 || (range4 && c->NP <= kMfma4MaxNP));
    int k = c->kernel_pref;
    if (k == WLD_KERNEL_AUTO) k = mfma_ok ? WLD_KERNEL_MFMA : WLD_KERNEL_VALU;
    if (k == WLD_KERNEL_MFMA && !(mfma_supported() && finite && maxabs > 0.0f))
        return fail(WLD_E_ARG, "MFMA kernel requested but weights are not finite/nonzero");
    if (k == WLD_KERNEL_MFMA && !mfma_fits)
        return fail(WLD_E_ARG, "MFMA kernel requested but %zu sequences exceed its int32 sums (max %zu)", N,
                    kMfmaMaxNP);
    c->kernel = k;
    c->safe = !finite;
    c->shift = 0;
    c->use_frag = false;
    if (k == WLD_KERNEL_MFMA) {
        // 3 planes when they hold every weight to 2^-19; else 4 (an explicit
        // MFMA request beyond 2^-12 keeps 4 planes and loses precision on the
        // smallest weights)
        c->fixed_planes = range3 || c->NP > kMfma4MaxNP ? 3 : 4;
        if (c->fixed_planes == 4 && c->opt_site_major)
            return fail(WLD_E_ARG, "the site-major MFMA kernel (WLD_OPT_MFMA_LAYOUT) multiplies 3 digit planes; "
                                   "these weights need 4");
        c->shift = weight_shift(maxabs, c->fixed_planes);
        WLD_TRY(ensure(c->planes, mfma_planes_bytes(c->LP, c->NP)));
        launch_mfma_prep(ptr<uint8_t>(c->site_ok), ptr<float>(c->w_pad), L, c->LP, c->NP, c->shift,
                         ptr<int8_t>(c->planes), c->stream);
        HIP_TRY(hipGetLastError());
        // fragment-major copy of the codes (1 KB contiguous per wave operand load);
        // WLD_OPT_MFMA_LAYOUT = 1 keeps the site-major reads (tests)
        c->use_frag = !c->opt_site_major;
        if (c->use_frag) {
            // two copies: the selector-coded one (A operands) and the
            // 0/1/2-coded one the B side reads raw
            WLD_TRY(ensure(c->frag, 2 * c->LP * c->NP));
            launch_frag(ptr<uint8_t>(c->codes), c->LP, c->NP, ptr<uint8_t>(c->frag), c->stream);
            HIP_TRY(hipGetLastError());
        }
    }
    HIP_TRY(hipEventRecord(c->ev[1], c->stream));

    c->has_map = site_map != nullptr;
    if (site_map) {
        std::vector<uint32_t> m(L);
        for (size_t i = 0; i < L; ++i) {
            if (site_map[i] > 0xFFFFFFFFull) return fail(WLD_E_ARG, "site_map[%zu] exceeds 32 bits", i);
            m[i] = (uint32_t)site_map[i];
        }
        WLD_TRY(ensure(c->site_map, std::max<size_t>(L, 1) * sizeof(uint32_t)));
        if (L) HIP_TRY(hipMemcpyAsync(c->site_map.p, m.data(), L * sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->wst = MfmaWeightStats{7, 1, {0, 0, 0}, {0, 0, 0, 0}};
    if (c->kernel == WLD_KERNEL_MFMA && mfma_weight_stats(ptr<int8_t>(c->planes), c->LP, c->NP, c->stream, &c->wst))
        return fail(WLD_E_HIP, "reading the weight-plane statistics failed");
    const unsigned all_planes = (1u << c->fixed_planes) - 1;
    c->plane_mask = c->kernel == WLD_KERNEL_MFMA && !c->opt_all_planes ? c->wst.plane_mask : all_planes;
    c->stats.load_ms = event_ms(c->ev[0], c->ev[1]);
    c->fp6_ok = c->fp6_better = c->fp6_tried = false;  // (fp6_prepare: at the first run that may use it)
    c->i8img_ok = false;  // (i8img_prepare: at the first pass that screens on i8)
    c->stats.mfma_planes = c->kernel == WLD_KERNEL_MFMA ? __builtin_popcount(c->plane_mask) : 0;
    c->stats.kernel = c->kernel;
    c->stats.weight_shift = c->shift;
    c->loaded = true;
    c->have_rows = false;
    c->tiles_lb = c->tiles_le = ~0u;
    // what a first run would otherwise build: the fp6 screen's operands (not
    // with WLD_OPT_SCREEN_FP6 0), lib.rs's lane-class layout (WLD_OPT_REF_SUMS),
    // the whole set's tile lists; a fresh context's first pass then costs
    // about a steady one (a run over a shard builds its own
    // lists on its first pass)
    if (c->opt_fp6 != 0) WLD_TRY(fp6_prepare(c));
    if (c->opt_ref_sums) WLD_TRY(ensure_ref_layout(c));
    {  // a run's pair count in O(1) (the per-chunk loop took microseconds per run);
       // up to 2^24 chunks (128 MB of prefix; ~1.48M sites), beyond that per run
        const uint32_t m = chunks_of(L), nr = chunk_rows_of(L);
        c->chunk_pairs_pre.assign(m <= (1u << 24) ? (size_t)m + 1 : 0, 0);
        for (uint32_t i = 0; i < m && m <= (1u << 24); ++i) {
            uint32_t row, col;
            chunk_of_linear_host(nr, i, row, col);
            c->chunk_pairs_pre[i + 1] = c->chunk_pairs_pre[i] + pairs_in_chunk(L, row, col);
        }
    }
    // the whole set's tile lists only where a whole-set run is possible (<=
    // 2^32 pairs, run_enqueue's limit; about 92,700 sites) and the lists stay
    // small (<= 2^22 tiles: 512 MB of candidate-list space at most); larger
    // sets run only as shards, whose first run builds its own lists
    {
        const uint64_t T_used = (L + kTile - 1) / kTile;
        if ((uint64_t)L * (L - 1) / 2 <= 0xFFFFFFFFull && T_used * (T_used + 1) / 2 <= (1ull << 22))
            WLD_TRY(build_tiles(c, 0, chunks_of(L)));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    return WLD_OK;
}

uint32_t chunk_rows_of(size_t L) { return (uint32_t)((L + kChunk - 1) / kChunk); }

uint64_t pairs_in_rows(size_t L, uint32_t rb, uint32_t re) {
    // pairs (a<b) with a in [rb*256, re*256) ∩ [0, L)
    uint64_t a0 = std::min<uint64_t>(L, (uint64_t)rb * kChunk), a1 = std::min<uint64_t>(L, (uint64_t)re * kChunk);
    uint64_t s = 0;
    // sum_{a=a0}^{a1-1} (L-1-a)
    if (a1 > a0) s = (a1 - a0) * (uint64_t)(L - 1) - (a1 - 1 + a0) * (a1 - a0) / 2;
    return s;
}

uint32_t chunks_of(size_t L) {
    const uint32_t n = chunk_rows_of(L);
    return n * (n + 1) / 2;
}

// (row, col) of linear chunk i: triu_index (lib.rs:623-632) in exact integers
void chunk_of_linear_host(uint32_t n, uint32_t i, uint32_t &row, uint32_t &col) {
    uint32_t rf = (uint32_t)((std::sqrt(8.0 * (double)i + 1.0) - 1.0) * 0.5);
    while ((uint64_t)(rf + 1) * (rf + 2) / 2 <= i) ++rf;
    while ((uint64_t)rf * (rf + 1) / 2 > i) --rf;
    row = n - rf - 1;
    col = row + i - rf * (rf + 1) / 2;
}

// pairs (a<b) of chunk (row, col): lib.rs:636-667's a/b loops
uint64_t pairs_in_chunk(size_t L, uint32_t row, uint32_t col) {
    auto side = [&](uint32_t r) -> uint64_t {
        const uint64_t lo = (uint64_t)r * kChunk;
        return lo >= L ? 0 : std::min<uint64_t>(L - lo, kChunk);
    };
    const uint64_t ra = side(row);
    return row == col ? ra * (ra ? ra - 1 : 0) / 2 : ra * side(col);
}

uint64_t pairs_in_chunks(size_t L, uint32_t lb, uint32_t le) {
    const uint32_t n = chunk_rows_of(L);
    uint64_t s = 0;
    for (uint32_t i = lb; i < le; ++i) {
        uint32_t r, c;
        chunk_of_linear_host(n, i, r, c);
        s += pairs_in_chunk(L, r, c);
    }
    return s;
}

// linear chunk range of chunk rows [rb, re): rows descend in linear order
void rows_to_linear(uint32_t n, uint32_t rb, uint32_t re, uint32_t &lb, uint32_t &le) {
    lb = re > rb ? chunk_linear(n, re - 1, re - 1) : 0;
    le = re > rb ? chunk_linear(n, rb, rb) + (n - rb) : 0;
}

// xcd_order and range_tiles: tile_order.hpp
using tile_order::xcd_order;

int build_tiles(wld_ctx *c, uint32_t lb, uint32_t le) {
    if (c->tiles_lb == lb && c->tiles_le == le && c->n_tiles) return WLD_OK;
    const uint32_t T_used = (uint32_t)((c->L + kTile - 1) / kTile);
    const uint32_t n = chunk_rows_of(c->L);
    std::vector<uint32_t> t = tile_order::range_tiles(n, T_used, lb, le);  // (ta, tb) order
    const uint32_t kS = tile_order::super_block_side((uint32_t)c->NP);
    // the fp6 screen's tile pairs (ordered as the tiles below, by first tile;
    // single tiles keep their flag through the ordering)
    std::vector<uint32_t> pl;
    if (T_used <= 0x7FFF && (int64_t)t.size() >= c->opt_fp6_pairs_min) {
        pl = tile_order::fp6_pair_list(t);
        if (!c->opt_tile_rows && pl.size() >= 2048) pl = xcd_order(pl, kS, ~tile_order::kSingleEntry);
    }
    // only with many rounds of resident tiles: whole super-blocks per XCD
    // leave up to one super-block of imbalance (C2's 528 tiles: +14%)
    if (!c->opt_tile_rows && t.size() >= 4096 && T_used < 65535) t = xcd_order(t, kS);
    c->n_tiles = (uint32_t)t.size();
    WLD_TRY(ensure(c->tiles, std::max<size_t>(t.size(), 1) * sizeof(uint32_t)));
    // screen candidates: 16 weight buckets of tiles, then of their sub-block bits
    WLD_TRY(ensure(c->cand, std::max<size_t>(t.size(), 1) * 32 * sizeof(uint32_t)));
    if (!t.empty())
        HIP_TRY(hipMemcpyAsync(c->tiles.p, t.data(), t.size() * sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
    c->f6_n_pairs = (uint32_t)pl.size();
    if (!pl.empty()) {
        WLD_TRY(ensure(c->f6_pairs, pl.size() * sizeof(uint32_t)));
        HIP_TRY(hipMemcpyAsync(c->f6_pairs.p, pl.data(), pl.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                               c->stream));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->tiles_lb = lb;
    c->tiles_le = le;
    return WLD_OK;
}

OrderArgs order_args(wld_ctx *c) {
    OrderArgs o;
    o.st_a = ptr<uint32_t>(c->st_a);
    o.st_b = ptr<uint32_t>(c->st_b);
    o.st_d = ptr<float>(c->st_d);
    o.st_dp = ptr<float>(c->st_dp);
    o.st_r2 = ptr<float>(c->st_r2);
    o.st_capacity = c->st_capacity;
    o.seg_cnt = ptr<uint8_t>(c->seg_cnt);
    o.seg_off = ptr<uint32_t>(c->seg_off);
    o.T = (uint32_t)(c->LP / kTile);
    o.chunk_total = ptr<uint32_t>(c->chunk_total);
    o.cursor = ptr<unsigned long long>(c->counters);
    o.chunk_left = c->prog_pass ? ptr<unsigned>(c->chunk_left) : nullptr;
    o.prog_n = c->prog_pass ? ptr<unsigned>(c->prog_n) : nullptr;
    o.prog_log = c->prog_pass ? c->d_plog : nullptr;
    o.L = (uint32_t)c->L;
    o.guard = reinterpret_cast<unsigned *>(c->d_hcnt + 4);
    return o;
}

// WLD_OPT_REF_SUMS: the codes and weights in the reference's lane-class order
// (pair_valu.hip), built once per load on first use
int ensure_ref_layout(wld_ctx *c) {
    if (c->have_ref) return WLD_OK;
    uint32_t tail = 0;
    ref_layout_dims(c->N, &c->ref_cls, &tail, &c->NPr);
    WLD_TRY(ensure(c->rcodes, c->LP * c->NPr));
    WLD_TRY(ensure(c->rw, c->NPr * sizeof(float)));
    launch_ref_layout(ptr<uint8_t>(c->codes), ptr<float>(c->w_pad), c->LP, c->NP, c->N, ptr<uint8_t>(c->rcodes),
                      ptr<float>(c->rw), c->stream);
    HIP_TRY(hipGetLastError());
    c->have_ref = true;
    return WLD_OK;
}

// How far (2x2-cell L1, fixed-point units of the weight planes) the
// reference's f32 sums can lie from the fixed-point sums the screen bounds:
// each weight is within 0.5 of w 2^shift (every sequence in one cell), and
// each of the four f32 sums within gamma_m sum|w| of its exact value
// (recursive summation: every term passes through at most m = N/8 + 16
// roundings — its lane chain, the horizontal sum, the scalar tail); the
// cells are n11 = SAB, n10 = SA - SAB, n01 = SB - SAB, n00 = T - SA - SB +
// SAB, so their L1 error is at most 9 times a sum's.  sum|q| <= sum_p 2^(8p)
// sum|d_p|.
double ref_extra_residual(const wld_ctx *c) {
    const double u = 0x1p-24, m = (double)(c->N / 8) + 16.0;
    const double gamma = m * u / (1.0 - m * u);
    double qsum = 0.0;
    for (int p = 0; p < 4; ++p) qsum += std::ldexp((double)c->wst.dsum[p], 8 * p);
    const double r = 9.0 * gamma * (qsum + 0.5 * (double)c->N) + 0.5 * (double)c->N;
    return r * (1.0 + 1e-9) + 1.0;  // slack for this evaluation's own rounding
}

// Enqueues the pair kernel(s) of a pass; *screened tells whether the MFMA
// screen ran (then ev[6] separates it from the candidate launch).
// With scan given, a screen fuses the run's chunk scan into its last
// workgroup or the candidate launch's (then the caller launches no scan).
int launch_pairs(wld_ctx *c, float thr, const OrderArgs &o, const DenseArgs *dense, bool *screened = nullptr,
                 const ScanArgs *scan = nullptr, bool *scan_fused = nullptr) {
    bool fused = false;  // the run's chunk scan ran inside a launch (the caller launches none)
    const uint32_t n = chunk_rows_of(c->L);
    bool sc = false;
    c->fp6_pass = false;
    c->stats.ref_sums = c->opt_ref_sums ? 1 : 0;
    c->ref_pairs_pass = false;
    ValuLaunch rv{};
    if (c->opt_ref_sums) {
        WLD_TRY(ensure_ref_layout(c));
        rv = ValuLaunch{ptr<uint8_t>(c->rcodes), ptr<float>(c->rw), ptr<uint8_t>(c->site_ok), ptr<uint32_t>(c->tiles),
                        c->n_tiles, nullptr, (uint32_t)c->L, (uint32_t)c->NPr, n, thr, c->safe, false, true,
                        c->ref_cls, (uint32_t)(c->N % 8)};
    }
    // reference order without a screen in front (no positive threshold, the
    // f32 kernel, dense stats, or the auto policy's full-kernel thresholds):
    // every tile on the reference-order f32 kernel
    const bool ref_screen = c->opt_ref_sums && c->kernel == WLD_KERNEL_MFMA && !dense && c->use_frag &&
                            c->opt_prefilter && thr > 0.0f && c->opt_screen != 0;
    // (a full run on the item kernel fuses the scan into its last workgroup)
    if (scan && !dense) rv.scan = *scan;
    if (c->opt_ref_sums && !ref_screen) {
        fused = launch_pair_valu(rv, o, dense, c->stream);
    } else if (c->kernel == WLD_KERNEL_MFMA) {
        MfmaLaunch m{};
        m.codes = ptr<uint8_t>(c->codes);
        m.frag = c->use_frag ? ptr<uint8_t>(c->frag) : nullptr;
        m.frag_b = c->use_frag ? ptr<uint8_t>(c->frag) + c->LP * c->NP : nullptr;
        m.wplanes = ptr<int8_t>(c->planes);
        m.tiles = ptr<uint32_t>(c->tiles);
        m.n_tiles = c->n_tiles;
        m.L = (uint32_t)c->L;
        m.NP = (uint32_t)c->NP;
        m.LP = (uint32_t)c->LP;
        m.n_chunk_rows = n;
        m.thr = thr;
        m.shift = c->shift;
        m.plane_mask = c->plane_mask;
        m.nonneg = c->wst.nonneg;
        // both need a positive threshold to reject anything
        m.prefilter = c->opt_prefilter && thr > 0.0f;
        // auto: below a threshold at which the screen left more than half the
        // tiles as candidates, every tile goes straight to the full kernel
        m.screen = m.prefilter && (c->opt_screen == 2 || c->opt_screen == 3 ||
                                   (c->opt_screen == 1 && thr > c->screen_bad_thr));
        // ... where the one-plane screen proved ineffective, the two-plane one
        // (>= 3 active planes), unless it proved ineffective too; in lib.rs's
        // order the exact candidate pairs instead (below)
        if (m.prefilter && !m.screen && c->opt_screen == 1 && !ref_screen && thr > c->screen2_bad_thr)
            m.screen = m.screen2 = true;
        if (c->opt_screen == 3) m.screen2 = true;
        if (m.screen2 && __builtin_popcount(c->plane_mask & 15) < 3) {
            m.screen2 = false;  // one or two active planes: the one-plane screen or the full kernel
            m.screen = c->opt_screen == 2 || c->opt_screen == 3;
        }
        c->screened2 = m.screen && m.screen2;
        for (int t = 0; t < 3; ++t) m.resid[t] = c->wst.resid[t];
        // the one-plane screen on fp6 x fp4 MFMA where the load allows it
        const bool fp6_auto = c->opt_fp6 == 1 || c->opt_fp6 == 3;
        m.fp6 = c->fp6_ok && (c->opt_fp6 == 2 || (fp6_auto && c->fp6_better && thr > c->fp6_bad_thr))
                    ? &c->f6 : nullptr;
        // auto: past a sixteenth of the tiles as candidates the fp6 screen
        // gives the pass up and run_complete re-runs it on the i8 screen (not
        // with per-chunk progress, which a re-run does not report again, nor
        // with a caller's count word, which a collective may read before the
        // re-run rewrites it)
        m.fp6_bail = fp6_auto && !c->prog_pass && !c->pend.count_out ? std::max<uint32_t>(c->n_tiles / 16, 1) : 0;
        m.f6_pairs = c->f6_n_pairs ? ptr<uint32_t>(c->f6_pairs) : nullptr;
        m.f6_n_pairs = c->f6_n_pairs;
        // the i8 one-plane screen on tile pairs (WLD_OPT_I8_PAIRS): its images
        // built at the first pass that needs them
        if (!dense && m.prefilter && m.screen && !m.screen2 && !m.fp6 && c->opt_i8_pairs && c->f6_n_pairs &&
            c->use_frag && c->wst.nonneg && c->NP <= 16384) {
            if (!c->i8img_ok) WLD_TRY(i8img_prepare(c));
            m.i8img = &c->i8s;
        }
        for (int p = 0; p < 4; ++p) m.dsum[p] = c->wst.dsum[p];
        m.cand_list = ptr<uint32_t>(c->cand);
        // this pass's candidate set (the scan zeroes the other one, enqueue_pass)
        unsigned long long *set = ptr<unsigned long long>(c->counters) + kCandSet0 + kCandSetWords * c->cand_set;
        m.cand_count = reinterpret_cast<unsigned *>(set);
        m.cand_work = reinterpret_cast<unsigned *>(ptr<unsigned long long>(c->counters) + 2) + 1;  // beside the ticket
        m.cand_buckets = reinterpret_cast<unsigned *>(set + 1);
        m.test_guard = c->opt_test_guard;
        if (scan && !dense) m.scan = *scan;
        RefRowsLaunch rr{};
        if (ref_screen) {
            m.ref_valu = &rv;
            m.r_extra_q = ref_extra_residual(c);
            // where the screen does not pay: every tile on all planes, the
            // pairs the bound cannot reject summed one by one in lib.rs's
            // order, unless that proved to be most pairs (then the full kernel)
            if (!m.screen && ((c->opt_screen == 1 && thr > c->ref_pairs_bad_thr) || c->opt_screen == 4)) {
                rr = RefRowsLaunch{ptr<uint8_t>(c->rcodes), ptr<float>(c->rw), (uint32_t)c->NPr, c->ref_cls,
                                   (uint32_t)(c->N % 8), n, thr, nullptr, nullptr, nullptr, ScanArgs{}};
                m.ref_rows = &rr;
                c->ref_pairs_pass = true;
            }
        }
        if (ref_screen && !m.screen && !m.ref_rows) {
            fused = launch_pair_valu(rv, o, nullptr, c->stream);  // the policy sends this threshold to the full kernel
        } else {
            sc = launch_pair_mfma(m, o, dense, c->stream, c->ev[6]);
            fused = sc && scan && !dense;  // (a screen's candidate launch, or the candidate pairs' compaction)
            c->fp6_pass = sc && m.fp6 && !m.screen2 && !m.ref_rows;  // (launch_pair_mfma's one-plane screen branch)
        }
    } else {
        launch_pair_valu(ValuLaunch{ptr<uint8_t>(c->codes), ptr<float>(c->w_pad), ptr<uint8_t>(c->site_ok),
                                    ptr<uint32_t>(c->tiles), c->n_tiles, nullptr, (uint32_t)c->L, (uint32_t)c->NP, n,
                                    thr, c->safe, c->opt_valu_plain, false, 0, 0},
                         o, dense, c->stream);
    }
    HIP_TRY(hipGetLastError());
    if (screened) *screened = sc;
    if (scan_fused) *scan_fused = fused;
    return WLD_OK;
}

}  // namespace

extern "C" {

const char *wld_version(void) { return "weightedld-amd 0.1.0 (gfx950)"; }

int wld_create(int device, wld_ctx **out) {
    if (!out) return fail(WLD_E_ARG, "wld_create: null out");
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) {
        (void)hipGetLastError();
        return fail(WLD_E_NODEV, "no HIP device visible (%s); the weightedld hot path runs only on a gfx950 GPU",
                    e == hipSuccess ? "0 devices" : hipGetErrorString(e));
    }
    if (device < 0 || device >= n) return fail(WLD_E_ARG, "device %d out of range (%d visible)", device, n);
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
        return fail(WLD_E_NODEV, "device %d is %s, not gfx950 (MI355X)", device, prop.gcnArchName);
    HIP_TRY(hipSetDevice(device));
    auto *c = new wld_ctx;
    c->device = device;
    hipError_t es = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
    c->stream = c->own_stream;
    if (es != hipSuccess) {
        delete c;
        return fail(WLD_E_HIP, "hipStreamCreate: %s", hipGetErrorString(es));
    }
    for (auto &ev : c->ev)
        if (hipEventCreate(&ev) != hipSuccess) {
            delete c;
            return fail(WLD_E_HIP, "hipEventCreate failed");
        }
    if (hipHostMalloc((void **)&c->h_cnt, 5 * sizeof(unsigned long long), hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess ||
        hipHostGetDevicePointer((void **)&c->d_hcnt, c->h_cnt, 0) != hipSuccess) {
        (void)hipGetLastError();
        delete c;
        return fail(WLD_E_HIP, "hipHostMalloc of the run counters failed");
    }
    *out = c;
    return WLD_OK;
}

int wld_create_multi(const int *devices, int n_devices, wld_ctx **out) {
    if (!out) return fail(WLD_E_ARG, "wld_create_multi: null out");
    *out = nullptr;
    if (!devices || n_devices < 1) return fail(WLD_E_ARG, "wld_create_multi: need at least one device");
    if (n_devices == 1) return wld_create(devices[0], out);  // a plain context: every entry point works
    auto *g = new wld_ctx;
    g->device = devices[0];
    for (int k = 0; k < n_devices; ++k) {
        wld_ctx *m = nullptr;
        const int st = wld_create(devices[k], &m);
        if (st != WLD_OK) {
            delete g;
            return st;
        }
        g->members.push_back(m);
    }
    *out = g;
    return WLD_OK;
}

int wld_n_devices(const wld_ctx *ctx) { return !ctx ? 0 : ctx->members.empty() ? 1 : (int)ctx->members.size(); }

void wld_destroy(wld_ctx *ctx) { delete ctx; }

int wld_set_kernel(wld_ctx *ctx, int kernel) {
    if (!ctx) return fail(WLD_E_ARG, "null context");
    for (wld_ctx *m : ctx->members) WLD_TRY(wld_set_kernel(m, kernel));
    if (kernel < WLD_KERNEL_AUTO || kernel > WLD_KERNEL_MFMA) return fail(WLD_E_ARG, "bad kernel id %d", kernel);
    if (kernel == WLD_KERNEL_MFMA && !mfma_supported()) return fail(WLD_E_ARG, "MFMA kernel not built");
    ctx->kernel_pref = kernel;
    return WLD_OK;
}

int wld_set_option(wld_ctx *c, int option, int64_t value) {
    if (!c) return fail(WLD_E_ARG, "null context");
    for (wld_ctx *m : c->members) WLD_TRY(wld_set_option(m, option, value));
    if (c->pend.active) return fail(WLD_E_STATE, "wld_set_option during a run");
    switch (option) {
        case WLD_OPT_PREFILTER: c->opt_prefilter = value != 0; break;
        case WLD_OPT_SCREEN:
            if (value < 0 || value > 4) return fail(WLD_E_ARG, "WLD_OPT_SCREEN takes 0 to 4");
            c->opt_screen = (int)value;
            c->screen_bad_thr = c->screen2_bad_thr = c->ref_pairs_bad_thr = c->fp6_bad_thr = -1.0f;
            c->fp6_good_thr = INFINITY;
            break;
        case WLD_OPT_TILE_ORDER:
            c->opt_tile_rows = value != 0;
            c->tiles_lb = c->tiles_le = ~0u;  // rebuild the list at the next run
            break;
        case WLD_OPT_ALL_PLANES:
            c->opt_all_planes = value != 0;
            if (c->loaded && c->kernel == WLD_KERNEL_MFMA)
                c->plane_mask = c->opt_all_planes ? (1u << c->fixed_planes) - 1 : c->wst.plane_mask;
            if (c->loaded) c->stats.mfma_planes = c->kernel == WLD_KERNEL_MFMA ? __builtin_popcount(c->plane_mask) : 0;
            break;
        case WLD_OPT_MFMA_LAYOUT: c->opt_site_major = value != 0; break;
        case WLD_OPT_VALU_PLAIN: c->opt_valu_plain = value != 0; break;
        case WLD_OPT_REF_SUMS:
            c->opt_ref_sums = value != 0;
            c->screen_bad_thr = c->screen2_bad_thr = c->ref_pairs_bad_thr = c->fp6_bad_thr = -1.0f;
            c->fp6_good_thr = INFINITY;  // the policy's break-even differs
            break;
        case WLD_OPT_STAGING_ROWS:
            if (value < 1) return fail(WLD_E_ARG, "WLD_OPT_STAGING_ROWS must be >= 1");
            c->opt_staging_rows = (uint64_t)value;
            break;
        case WLD_OPT_HOST_BATCH_PAIRS:
            if (value < 1) return fail(WLD_E_ARG, "WLD_OPT_HOST_BATCH_PAIRS must be >= 1");
            c->opt_host_batch_pairs = (uint64_t)value;
            break;
        case WLD_OPT_FUSED_SCAN: c->opt_fused_scan = value != 0; break;
        case WLD_OPT_I8_PAIRS: c->opt_i8_pairs = value != 0; break;
        case WLD_OPT_TEST_GUARD: c->opt_test_guard = value != 0; break;
        case WLD_OPT_FP6_PAIRS_MIN_TILES:
            if (value < 0) return fail(WLD_E_ARG, "WLD_OPT_FP6_PAIRS_MIN_TILES must be >= 0");
            c->opt_fp6_pairs_min = value;
            c->tiles_lb = c->tiles_le = ~0u;  // rebuild the lists at the next run
            break;
        case WLD_OPT_SCREEN_FP6:
            if (value < 0 || value > 3) return fail(WLD_E_ARG, "WLD_OPT_SCREEN_FP6 takes 0 to 3");
            c->opt_fp6 = (int)value;
            c->screen_bad_thr = c->screen2_bad_thr = c->ref_pairs_bad_thr = c->fp6_bad_thr = -1.0f;
            c->fp6_good_thr = INFINITY;  // another screen's break-even
            break;
        default: return fail(WLD_E_ARG, "unknown option %d", option);
    }
    return WLD_OK;
}

int wld_get_option(wld_ctx *c, int option, int64_t *value) {
    if (!c || !value) return fail(WLD_E_ARG, "null argument");
    switch (option) {
        case WLD_OPT_PREFILTER: *value = c->opt_prefilter; break;
        case WLD_OPT_SCREEN: *value = c->opt_screen; break;
        case WLD_OPT_TILE_ORDER: *value = c->opt_tile_rows; break;
        case WLD_OPT_ALL_PLANES: *value = c->opt_all_planes; break;
        case WLD_OPT_MFMA_LAYOUT: *value = c->opt_site_major; break;
        case WLD_OPT_VALU_PLAIN: *value = c->opt_valu_plain; break;
        case WLD_OPT_REF_SUMS: *value = c->opt_ref_sums; break;
        case WLD_OPT_STAGING_ROWS: *value = (int64_t)c->opt_staging_rows; break;
        case WLD_OPT_HOST_BATCH_PAIRS: *value = (int64_t)c->opt_host_batch_pairs; break;
        case WLD_OPT_FUSED_SCAN: *value = c->opt_fused_scan; break;
        case WLD_OPT_TEST_GUARD: *value = c->opt_test_guard; break;
        case WLD_OPT_FP6_PAIRS_MIN_TILES: *value = c->opt_fp6_pairs_min; break;
        case WLD_OPT_SCREEN_FP6: *value = c->opt_fp6; break;
        case WLD_OPT_I8_PAIRS: *value = c->opt_i8_pairs; break;
        default: return fail(WLD_E_ARG, "unknown option %d", option);
    }
    return WLD_OK;
}

int wld_load(wld_ctx *c, const uint8_t *sites, size_t n_sites, size_t n_seqs, const uint64_t *site_map,
             const float *weights) {
    if (c && !c->members.empty()) {
        // every device gets the whole input (replicated; it is small next to
        // the pair space), loaded concurrently
        const size_t G = c->members.size();
        std::vector<int> st(G, WLD_OK);
        std::vector<std::string> msg(G);
        std::vector<std::thread> th;
        for (size_t k = 0; k < G; ++k)
            th.emplace_back([&, k] {
                st[k] = wld_load(c->members[k], sites, n_sites, n_seqs, site_map, weights);
                if (st[k] != WLD_OK) msg[k] = wld_last_error();
            });
        for (auto &t : th) t.join();
        for (size_t k = 0; k < G; ++k)
            if (st[k] != WLD_OK) return fail(st[k], "device %d: %s", c->members[k]->device, msg[k].c_str());
        c->stats = c->members[0]->stats;
        return WLD_OK;
    }
    WLD_TRY(set_dev(c));
    if ((!sites && n_sites * n_seqs) || (!weights && n_seqs)) return fail(WLD_E_ARG, "wld_load: null input");
    if (n_sites >= (1u << 16) * (size_t)kTile) return fail(WLD_E_ARG, "n_sites %zu too large", n_sites);
    c->loaded = false;
    c->prepass_loaded = false;
    c->L = n_sites;
    c->N = n_seqs;
    WLD_TRY(ensure(c->raw, n_sites * n_seqs));
    WLD_TRY(ensure(c->wraw, n_seqs * sizeof(float)));
    if (n_sites * n_seqs)
        HIP_TRY(hipMemcpyAsync(c->raw.p, sites, n_sites * n_seqs, hipMemcpyHostToDevice, c->stream));
    if (n_seqs) HIP_TRY(hipMemcpyAsync(c->wraw.p, weights, n_seqs * sizeof(float), hipMemcpyHostToDevice, c->stream));
    return common_load(c, ptr<uint8_t>(c->raw), ptr<float>(c->wraw), site_map);
}

int wld_load_device(wld_ctx *c, const void *d_sites, size_t n_sites, size_t n_seqs, const uint64_t *site_map,
                    const void *d_weights) {
    WLD_TRY(set_dev(c));
    if ((!d_sites && n_sites * n_seqs) || (!d_weights && n_seqs)) return fail(WLD_E_ARG, "wld_load_device: null input");
    if (n_sites >= (1u << 16) * (size_t)kTile) return fail(WLD_E_ARG, "n_sites %zu too large", n_sites);
    c->loaded = false;
    c->prepass_loaded = false;
    c->L = n_sites;
    c->N = n_seqs;
    return common_load(c, (const uint8_t *)d_sites, (const float *)d_weights, site_map);
}

namespace {
// wld_load_filtered[_device]: site stats on every raw site, kept-site map on
// the host (one byte per site back), Henikoff on the kept sites, then the
// common load of the kept set straight from the raw rows.
int load_filtered(wld_ctx *c, const uint8_t *d_raw, size_t n_sites, size_t n_seqs, const uint64_t *raw_map,
                  float min_acgt, float min_minor, float max_minor, int unweighted, size_t *n_kept) {
    if (n_sites >= (1u << 31)) return fail(WLD_E_ARG, "n_sites %zu too large", n_sites);
    c->loaded = false;
    c->prepass_loaded = false;
    const size_t L0 = n_sites, N = n_seqs;
    // main.rs:139: ceil(min_acgt * n_seqs) in f32, `as usize` saturating at 0 (host.cpp)
    const float cnt = std::ceil(min_acgt * (float)N);
    const uint32_t min_acgt_cnt = cnt <= 0.0f ? 0u : (uint32_t)std::min<double>(cnt, 4294967295.0);
    WLD_TRY(ensure(c->keep, std::max<size_t>(L0, 1)));
    WLD_TRY(ensure(c->htab, std::max<size_t>(L0, 1) * 6 * sizeof(float)));
    HIP_TRY(hipEventRecord(c->ev[0], c->stream));
    launch_site_stats(d_raw, L0, N, min_acgt_cnt, min_minor, max_minor, ptr<uint8_t>(c->keep), ptr<float>(c->htab),
                      c->stream);
    HIP_TRY(hipGetLastError());
    std::vector<uint8_t> keep(L0);
    if (L0) HIP_TRY(hipMemcpyAsync(keep.data(), c->keep.p, L0, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->kept_map.clear();
    std::vector<uint32_t> idx;
    for (size_t i = 0; i < L0; ++i)
        if (keep[i]) {
            c->kept_map.push_back(raw_map ? raw_map[i] : (uint64_t)i);
            idx.push_back((uint32_t)i);
        }
    const size_t L = idx.size();
    if (L >= (1u << 16) * (size_t)kTile) return fail(WLD_E_ARG, "%zu kept sites: too many", L);
    WLD_TRY(ensure(c->site_index, std::max<size_t>(L, 1) * sizeof(uint32_t)));
    if (L) HIP_TRY(hipMemcpyAsync(c->site_index.p, idx.data(), L * sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
    WLD_TRY(ensure(c->wraw, std::max<size_t>(N, 1) * sizeof(float)));
    if (unweighted)
        launch_fill_ones(ptr<float>(c->wraw), N, c->stream);
    else {
        WLD_TRY(ensure(c->htab_kept, std::max<size_t>(L, 1) * 6 * sizeof(float)));
        launch_henikoff(d_raw, ptr<uint32_t>(c->site_index), L, N, ptr<float>(c->htab), ptr<float>(c->htab_kept),
                        ptr<float>(c->wraw), c->stream);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(c->ev[1], c->stream));
    HIP_TRY(hipEventSynchronize(c->ev[1]));
    const double prepass_ms = event_ms(c->ev[0], c->ev[1]);
    c->L = L;
    c->N = N;
    WLD_TRY(common_load(c, d_raw, ptr<float>(c->wraw), c->kept_map.data(), ptr<uint32_t>(c->site_index)));
    c->stats.load_ms += prepass_ms;
    c->prepass_loaded = true;
    if (n_kept) *n_kept = L;
    return WLD_OK;
}
}  // namespace

int wld_load_filtered(wld_ctx *c, const uint8_t *sites, size_t n_sites, size_t n_seqs, const uint64_t *site_map,
                      float min_acgt, float min_minor, float max_minor, int unweighted, size_t *n_kept) {
    WLD_TRY(set_dev(c));
    if (!sites && n_sites * n_seqs) return fail(WLD_E_ARG, "wld_load_filtered: null input");
    WLD_TRY(ensure(c->raw, std::max<size_t>(n_sites * n_seqs, 1)));
    if (n_sites * n_seqs)
        HIP_TRY(hipMemcpyAsync(c->raw.p, sites, n_sites * n_seqs, hipMemcpyHostToDevice, c->stream));
    return load_filtered(c, ptr<uint8_t>(c->raw), n_sites, n_seqs, site_map, min_acgt, min_minor, max_minor,
                         unweighted, n_kept);
}

int wld_load_filtered_device(wld_ctx *c, const void *d_sites, size_t n_sites, size_t n_seqs,
                             const uint64_t *site_map, float min_acgt, float min_minor, float max_minor,
                             int unweighted, size_t *n_kept) {
    WLD_TRY(set_dev(c));
    if (!d_sites && n_sites * n_seqs) return fail(WLD_E_ARG, "wld_load_filtered_device: null input");
    return load_filtered(c, (const uint8_t *)d_sites, n_sites, n_seqs, site_map, min_acgt, min_minor, max_minor,
                         unweighted, n_kept);
}

int wld_weights_copy(wld_ctx *c, float *out) {
    WLD_TRY(set_dev(c));
    if (!c->prepass_loaded) return fail(WLD_E_STATE, "wld_weights_copy before wld_load_filtered");
    if (!out && c->N) return fail(WLD_E_ARG, "wld_weights_copy: null output");
    if (c->N) HIP_TRY(hipMemcpyAsync(out, c->wraw.p, c->N * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return WLD_OK;
}

int wld_site_map_copy(wld_ctx *c, uint64_t *out) {
    if (!c) return fail(WLD_E_ARG, "null context");
    if (!c->prepass_loaded) return fail(WLD_E_STATE, "wld_site_map_copy before wld_load_filtered");
    if (!out && !c->kept_map.empty()) return fail(WLD_E_ARG, "wld_site_map_copy: null output");
    std::copy(c->kept_map.begin(), c->kept_map.end(), out);
    return WLD_OK;
}

uint32_t wld_chunk_rows(size_t n_sites) { return chunk_rows_of(n_sites); }

int wld_shard_chunk_rows(size_t n_sites, int n_shards, int shard, uint32_t *begin, uint32_t *end) {
    if (n_shards < 1 || shard < 0 || shard >= n_shards || !begin || !end)
        return fail(WLD_E_ARG, "bad shard %d/%d", shard, n_shards);
    const uint32_t n = chunk_rows_of(n_sites);
    const uint64_t total = pairs_in_rows(n_sites, 0, n);
    // boundaries: first chunk row where the cumulative pair count reaches k/n_shards
    auto boundary = [&](int k) -> uint32_t {
        if (k <= 0) return 0;
        if (k >= n_shards) return n;
        const long double target = (long double)total * k / n_shards;
        uint32_t r = 0;
        while (r < n && (long double)pairs_in_rows(n_sites, 0, r + 1) <= target) ++r;
        // pick the closer of r and r+1
        if (r < n) {
            long double lo = (long double)pairs_in_rows(n_sites, 0, r), hi = (long double)pairs_in_rows(n_sites, 0, r + 1);
            if (hi - target < target - lo) ++r;
        }
        return r;
    };
    *begin = boundary(shard);
    *end = boundary(shard + 1);
    if (*end < *begin) *end = *begin;
    return WLD_OK;
}

uint32_t wld_chunks(size_t n_sites) { return chunks_of(n_sites); }

uint64_t wld_pairs_in_chunks(size_t n_sites, uint32_t begin, uint32_t end) {
    return pairs_in_chunks(n_sites, begin, std::min<uint32_t>(end, chunks_of(n_sites)));
}

int wld_shard_chunks(size_t n_sites, int n_shards, int shard, uint32_t *begin, uint32_t *end) {
    if (n_shards < 1 || shard < 0 || shard >= n_shards || !begin || !end)
        return fail(WLD_E_ARG, "bad shard %d/%d", shard, n_shards);
    const uint32_t m = chunks_of(n_sites), n = chunk_rows_of(n_sites);
    std::vector<uint64_t> pre(m + 1, 0);  // pairs in linear chunks [0, i)
    for (uint32_t i = 0; i < m; ++i) {
        uint32_t r, c;
        chunk_of_linear_host(n, i, r, c);
        pre[i + 1] = pre[i] + pairs_in_chunk(n_sites, r, c);
    }
    // boundary j: the linear chunk whose prefix is closest to j/n_shards of the total
    auto boundary = [&](int j) -> uint32_t {
        if (j <= 0) return 0;
        if (j >= n_shards) return m;
        const long double target = (long double)pre[m] * j / n_shards;
        uint32_t i = (uint32_t)(std::upper_bound(pre.begin(), pre.end(), (uint64_t)target) - pre.begin()) - 1;
        if (i < m && (long double)pre[i + 1] - target < target - (long double)pre[i]) ++i;
        return i;
    };
    // shard k takes the k-th range from the END of the linear order, so shards
    // concatenate in descending shard order as with wld_shard_chunk_rows
    *begin = boundary(n_shards - 1 - shard);
    *end = boundary(n_shards - shard);
    if (*end < *begin) *end = *begin;
    return WLD_OK;
}

namespace {
int ensure_outputs(wld_ctx *c, uint64_t rows) {
    rows = std::max<uint64_t>(rows, 1);
    WLD_TRY(ensure(c->out_a, rows * 4));
    WLD_TRY(ensure(c->out_b, rows * 4));
    WLD_TRY(ensure(c->out_d, rows * 4));
    WLD_TRY(ensure(c->out_dp, rows * 4));
    WLD_TRY(ensure(c->out_r2, rows * 4));
    return WLD_OK;
}

int grow_staging(wld_ctx *c, uint64_t cap) {
    cap = std::max<uint64_t>(cap, 1);
    if (c->st_capacity >= cap) return WLD_OK;
    WLD_TRY(ensure(c->st_a, cap * 4));
    WLD_TRY(ensure(c->st_b, cap * 4));
    WLD_TRY(ensure(c->st_d, cap * 4));
    WLD_TRY(ensure(c->st_dp, cap * 4));
    WLD_TRY(ensure(c->st_r2, cap * 4));
    c->st_capacity = cap;
    return WLD_OK;
}

// One pass of a run, enqueued on the context's stream with no host wait:
// run-state init, the pair kernel, then the chunk scan, which leaves
// {staging cursor, row total} in the mapped host counters (and the total in
// the caller's device word, if given).
int enqueue_pass(wld_ctx *c) {
    const RunPending &r = c->pend;
    if (c->times_pending) {  // the last pass's times were never asked for: its events are re-recorded now
        c->times_pending = false;
        c->stats.pair_kernel_ms = c->stats.order_ms = c->stats.screen_ms = -1.0;
    }
    const uint32_t lin_count = r.lin_end - r.lin_begin;
    // The chunk scan of every completed run leaves the cursor and its chunk
    // totals at 0, and every computed tile writes all of its segment counts,
    // so the init kernel runs only after (re)allocation or a failed run.
    if (c->run_dirty) {
        const uint32_t n = chunk_rows_of(c->L);
        launch_run_init(ptr<unsigned long long>(c->counters), ptr<uint32_t>(c->chunk_total), n * (n + 1) / 2,
                        c->stream);
        HIP_TRY(hipGetLastError());
    }
    c->run_dirty = true;  // until run_complete has seen this pass's scan
    // the reference-order layout is built (once per load) before the pass's
    // first event, so its kernel never lands in the pair phase's time
    if (c->opt_ref_sums && c->n_tiles) WLD_TRY(ensure_ref_layout(c));
    const OrderArgs o = order_args(c);
    // counters: {cursor, total, {ticket, work}, candidate set 0, candidate set 1}
    // (kernels.hpp).  The pass appends to set cand_set; its scan reads that
    // set's counts and zeroes the other one, which the next pass then uses —
    // no kernel of this pass can read a count its own scan has reset.
    unsigned long long *cn = ptr<unsigned long long>(c->counters);
    unsigned long long *cur = cn + kCandSet0 + kCandSetWords * c->cand_set;
    unsigned long long *nxt = cn + kCandSet0 + kCandSetWords * (c->cand_set ^ 1);
    ScanArgs sa{ptr<uint32_t>(c->chunk_total), r.lin_begin, lin_count, ptr<uint32_t>(c->chunk_base), cn + 1, cn,
                c->d_hcnt, r.count_out, cn + kCursorSeen, reinterpret_cast<unsigned *>(cur), reinterpret_cast<unsigned *>(nxt),
                reinterpret_cast<unsigned *>(nxt + 1), reinterpret_cast<unsigned *>(cn + 2)};
    c->h_cnt[0] = c->h_cnt[1] = lin_count ? ~0ull : 0ull;
    c->h_cnt[2] = c->h_cnt[3] = 0;
    c->h_cnt[4] = 0;  // the guard word
    HIP_TRY(hipEventRecord(c->ev[2], c->stream));
    c->screened = c->screened2 = false;
    // the scan is fused into the launch after a screen for ranges up to 4096
    // chunks (C4: 3,160, ~10 us in one 256-thread workgroup); a larger range
    // (C5: 19,306 chunks, ~70 us fused) gets the 1024-thread scan kernel
    const bool fuse_scan = c->opt_fused_scan && lin_count && lin_count <= 4096;
    bool scan_fused = false;
    if (c->n_tiles)
        WLD_TRY(launch_pairs(c, r.thr, o, nullptr, &c->screened, fuse_scan ? &sa : nullptr, &scan_fused));
    if (lin_count) c->cand_set ^= 1;  // this pass's scan (fused or below) zeroes the other set
    HIP_TRY(hipEventRecord(c->ev[3], c->stream));
    if (lin_count && !scan_fused) {  // else the last workgroup of the pair launch ran it
        sa.ticket = nullptr;
        launch_chunk_scan(sa, c->stream);
        HIP_TRY(hipGetLastError());
    } else if (!lin_count && r.count_out) {
        HIP_TRY(hipMemsetAsync(r.count_out, 0, sizeof(unsigned long long), c->stream));
    }
    // (a scan fused into the pair launch ends with it: ev[3] marks both, one
    // event record fewer per pass)
    c->ev_end = scan_fused ? 3 : 4;
    if (!scan_fused) HIP_TRY(hipEventRecord(c->ev[4], c->stream));
    c->gather_cap = 0;
    if (c->spec_gather && lin_count) {
        // outputs for a quarter more rows than the last run's (the scan's
        // count decides; more than that and run_complete gathers again)
        const uint64_t cap = std::min<uint64_t>(c->st_capacity, c->rows + c->rows / 4 + 4096);
        WLD_TRY(ensure_outputs(c, cap));
        launch_gather(o, ptr<uint32_t>(c->chunk_base), r.lin_begin, lin_count, chunk_rows_of(c->L), (uint32_t)c->L, 0,
                      cn, c->out_a.bytes / 4, c->has_map ? ptr<uint32_t>(c->site_map) : nullptr,
                      ptr<uint32_t>(c->out_a), ptr<uint32_t>(c->out_b), ptr<float>(c->out_d), ptr<float>(c->out_dp),
                      ptr<float>(c->out_r2), c->stream);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(c->ev[5], c->stream));
        c->gather_cap = c->out_a.bytes / 4;
    }
    return WLD_OK;
}

// The fp6 screen's eligibility for this pass, decided from a sample (auto,
// WLD_OPT_SCREEN_FP6 1) instead of a given-up pass: on linkage-structured
// data the fp6 rounding leaves nearly every tile a candidate, and a pass that
// gives up past a sixteenth of them still costs several times a screen
// (DESIGN.md §4.1).  Every stride-th entry of the screen's list (about 1/64
// of it) is screened, counting only; past a sixteenth of the sampled tiles as
// candidates the threshold (and any lower one) goes to the i8 screen, else it
// (and any higher one) stays on fp6 with no further sample.  Small lists
// (fewer than 2,048 tiles) take the pass itself as the test, as before.
// Only where the pass would run the one-plane screen (launch_pairs: the
// screen policy, no dense stats); on the context's own stream when the
// caller lent it one and the fp6 operands were built before this run (the
// probe reads only them), so the read-back does not wait for the caller's
// earlier work on the borrowed stream.
int fp6_sample(wld_ctx *c, float thr, bool operands_fresh) {
    if (c->opt_fp6 != 1 || !c->fp6_ok || !c->fp6_better || !(thr > c->fp6_bad_thr) || thr >= c->fp6_good_thr)
        return WLD_OK;
    if (c->kernel != WLD_KERNEL_MFMA || !c->use_frag || !c->opt_prefilter || !(thr > 0.0f) || c->opt_screen == 0 ||
        c->n_tiles < 2048)
        return WLD_OK;
    if (!(c->opt_screen == 2 || c->opt_screen == 3 || (c->opt_screen == 1 && thr > c->screen_bad_thr)))
        return WLD_OK;  // no one-plane screen at this threshold: nothing to decide
    const hipStream_t s = !operands_fresh && c->own_stream ? c->own_stream : c->stream;
    WLD_TRY(ensure(c->fp6_probe_buf, 2 * sizeof(unsigned)));
    MfmaLaunch m{};
    m.wplanes = ptr<int8_t>(c->planes);
    m.tiles = ptr<uint32_t>(c->tiles);
    m.n_tiles = c->n_tiles;
    m.L = (uint32_t)c->L;
    m.NP = (uint32_t)c->NP;
    m.LP = (uint32_t)c->LP;
    m.n_chunk_rows = chunk_rows_of(c->L);
    m.thr = thr;
    m.nonneg = c->wst.nonneg;
    m.fp6 = &c->f6;
    m.f6_pairs = c->f6_n_pairs ? ptr<uint32_t>(c->f6_pairs) : nullptr;
    m.f6_n_pairs = c->f6_n_pairs;
    const uint32_t entries = m.f6_pairs ? m.f6_n_pairs : m.n_tiles;
    const uint32_t stride = std::max<uint32_t>(1, std::min<uint32_t>(64, entries / 256));
    launch_fp6_probe(m, ptr<unsigned>(c->fp6_probe_buf), stride, s);
    HIP_TRY(hipGetLastError());
    unsigned h[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(h, c->fp6_probe_buf.p, sizeof(h), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    c->fp6_sampled = true;
    if ((uint64_t)h[0] * 16 > h[1])
        c->fp6_bad_thr = std::max(c->fp6_bad_thr, thr);
    else
        c->fp6_good_thr = std::min(c->fp6_good_thr, thr);
    return WLD_OK;
}

// Phase 1 of a run over linear chunks [lin_begin, lin_end): sizing, then the
// first pass, enqueued.  Staging starts at min(pairs, 32M rows); the pair
// kernels count every passing row but store only below capacity, so an
// overflow is detected from the cursor in run_complete and the pass re-run
// once with staging of the exact size.
int run_enqueue(wld_ctx *c, float thr, uint32_t lin_begin, uint32_t lin_end, unsigned long long *count_out) {
    const uint32_t n = chunk_rows_of(c->L);
    c->have_rows = false;
    c->pend.active = false;
    const bool fp6_fresh = !c->fp6_tried && c->opt_fp6 != 0;
    if (fp6_fresh) WLD_TRY(fp6_prepare(c));
    WLD_TRY(build_tiles(c, lin_begin, lin_end));
    c->fp6_sampled = false;
    WLD_TRY(fp6_sample(c, thr, fp6_fresh));
    const uint64_t pairs = c->chunk_pairs_pre.size() > lin_end
                               ? c->chunk_pairs_pre[lin_end] - c->chunk_pairs_pre[lin_begin]
                               : pairs_in_chunks(c->L, lin_begin, lin_end);
    const uint32_t T = (uint32_t)(c->LP / kTile);
    const uint32_t n_chunks = n * (n + 1) / 2;
    if (pairs > 0xFFFFFFFFull)
        return fail(WLD_E_ARG, "shard has %llu pairs; > 2^32 per device not supported (shard over more devices)",
                    (unsigned long long)pairs);
    WLD_TRY(grow_staging(c, std::min<uint64_t>(pairs, c->opt_staging_rows)));
    WLD_TRY(ensure(c->seg_cnt, c->LP * T));
    WLD_TRY(ensure(c->seg_off, c->LP * T * sizeof(uint32_t)));
    const size_t ct_bytes = c->chunk_total.bytes, cn_bytes = c->counters.bytes;
    WLD_TRY(ensure(c->chunk_total, std::max<size_t>(n_chunks, 1) * sizeof(uint32_t)));
    WLD_TRY(ensure(c->chunk_base, std::max<size_t>(n_chunks, 1) * sizeof(uint32_t)));
    WLD_TRY(ensure(c->counters, kCounterWords * sizeof(unsigned long long)));
    if (c->chunk_total.bytes != ct_bytes || c->counters.bytes != cn_bytes) c->run_dirty = true;  // fresh memory
    c->pend = RunPending{true, thr, lin_begin, lin_end, pairs, count_out};
    c->prog_pass = false;
    if (c->on_chunk && lin_end > lin_begin) {
        // per-chunk progress: countdowns of the range's chunks, an empty log
        const uint32_t cnt = lin_end - lin_begin;
        WLD_TRY(ensure(c->chunk_left, std::max<size_t>(n_chunks, 1) * sizeof(unsigned)));
        WLD_TRY(ensure(c->prog_n, sizeof(unsigned)));
        if (c->plog_cap < cnt) {
            if (c->h_plog) (void)hipHostFree(c->h_plog);
            c->h_plog = c->d_plog = nullptr;
            c->plog_cap = 0;
            HIP_TRY(hipHostMalloc((void **)&c->h_plog, (size_t)cnt * sizeof(unsigned long long),
                                  hipHostMallocMapped | hipHostMallocCoherent));
            HIP_TRY(hipHostGetDevicePointer((void **)&c->d_plog, c->h_plog, 0));
            c->plog_cap = cnt;
        }
        memset(c->h_plog, 0xFF, (size_t)cnt * sizeof(unsigned long long));
        launch_progress_init(ptr<unsigned>(c->chunk_left), lin_begin, cnt, n, (uint32_t)c->L, ptr<unsigned>(c->prog_n),
                             c->stream);
        HIP_TRY(hipGetLastError());
        c->prog_pass = true;
    }
    return enqueue_pass(c);
}

// The progress log of a pass with per-chunk progress: every chunk pair count
// logged so far, in slot order, to on_chunk (on the calling thread), polled
// while the pass runs; then the rest once it has completed.  Progress is a
// report, not a result: entries still missing once the pass has completed
// are reported from the chunk pair counts the host knows rather than failing
// the run, and counted in wld_run_stats.progress_filled — a pass that
// completes logs every chunk (a refused tile fails the run at check_guard),
// so a nonzero count is a lost tile_done count, which the tests look for.
int drain_progress(wld_ctx *c, uint32_t lin_begin, uint32_t n_chunks) {
    uint32_t seen = 0;
    auto drain = [&] {
        while (seen < n_chunks) {
            const unsigned long long v = __atomic_load_n(&c->h_plog[seen], __ATOMIC_ACQUIRE);
            if (v == ~0ull) break;
            (*c->on_chunk)(v);
            ++seen;
        }
    };
    for (;;) {
        const hipError_t q = hipEventQuery(c->ev[c->ev_end]);  // the pass's end (the stream may hold later work)
        drain();
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) HIP_TRY(q);
        std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
    // the pass has completed: every chunk's entry is written (system-scope
    // stores); allow the last ones a moment to land
    for (int spin = 0; seen < n_chunks && spin < 100000; ++spin) drain();
    if (seen < n_chunks) {
        // the logged chunks' pairs, then the pairs of the chunks whose entries
        // did not arrive, one report each (the sum is the range's pairs)
        uint64_t logged = 0;
        for (uint32_t k = 0; k < seen; ++k) logged += c->h_plog[k];
        uint64_t rest = pairs_in_chunks(c->L, lin_begin, lin_begin + n_chunks) - std::min<uint64_t>(
                            logged, pairs_in_chunks(c->L, lin_begin, lin_begin + n_chunks));
        const uint32_t missing = n_chunks - seen;
        c->stats.progress_filled += missing;
        for (uint32_t k = 0; k < missing; ++k) {
            const uint64_t v = rest / (missing - k);
            (*c->on_chunk)(v);
            rest -= v;
        }
    }
    return WLD_OK;
}

// The kernels' guard word (OrderArgs::guard) after a completed phase: nonzero
// when a kernel refused an out-of-range index (a candidate entry or tile, a
// staged pair, a gather destination) instead of reading or writing through
// it.  The run is then wrong, not just slow: WLD_E_STATE, and the next run
// starts from re-initialised run state.
int check_guard(wld_ctx *c, const char *phase) {
    const unsigned g = (unsigned)__atomic_load_n(&c->h_cnt[4], __ATOMIC_ACQUIRE);
    if (!g) return WLD_OK;
    c->run_dirty = true;
    c->have_rows = false;
    return fail(WLD_E_STATE, "internal: the %s refused an out-of-range index (guard 0x%x: %s%s%s%s%s); no rows", phase,
                g, g & kGuardEntry ? "candidate entry " : "", g & kGuardTile ? "tile " : "",
                g & kGuardPair ? "staged pair " : "", g & kGuardSlice ? "candidate slice " : "",
                g & kGuardGather ? "gather destination" : "");
}

// Phase 2: one host wait, the overflow re-run if needed, then (only when rows
// passed) the reference-order gather.
int run_complete(wld_ctx *c, uint64_t *n_rows) {
    if (!c->pend.active) return fail(WLD_E_STATE, "no run in flight");
    c->pend.active = false;
    const RunPending r = c->pend;
    const uint32_t n = chunk_rows_of(c->L);
    const uint32_t lin_count = r.lin_end - r.lin_begin;
    unsigned long long h[4] = {0, 0, 0, 0};
    bool regrown = false, abandoned = false;
    for (;;) {
        if (c->prog_pass) {
            c->prog_pass = false;  // a re-run after a staging overflow does not report again
            WLD_TRY(drain_progress(c, r.lin_begin, lin_count));
        }
        // the pass's end, not the stream's: on a shared stream (wld_set_stream)
        // the next context's run may already be queued behind it
        HIP_TRY(hipEventSynchronize(c->ev[c->gather_cap ? 5 : c->ev_end]));
        WLD_TRY(check_guard(c, c->gather_cap ? "pair phase or reference-order gather" : "pair phase"));
        c->run_dirty = false;  // the pass completed: its scan cleaned the run state
        h[0] = __atomic_load_n(&c->h_cnt[0], __ATOMIC_ACQUIRE);
        h[1] = __atomic_load_n(&c->h_cnt[1], __ATOMIC_ACQUIRE);
        h[2] = __atomic_load_n(&c->h_cnt[2], __ATOMIC_ACQUIRE);
        h[3] = __atomic_load_n(&c->h_cnt[3], __ATOMIC_ACQUIRE);
        if (h[2] & kAbandonBit) {
            // the fp6 screen gave the pass up: this threshold (and any lower
            // one) screens on i8 from now on, this pass included
            if (abandoned) return fail(WLD_E_HIP, "internal: a re-run pass was abandoned again");
            abandoned = true;
            c->fp6_bad_thr = std::max(c->fp6_bad_thr, r.thr);
            WLD_TRY(enqueue_pass(c));
            continue;
        }
        if (h[0] <= c->st_capacity) break;
        if (regrown) return fail(WLD_E_HIP, "internal: staging overflow after resize");
        regrown = true;
        WLD_TRY(grow_staging(c, h[0]));
        WLD_TRY(enqueue_pass(c));
    }
    const uint64_t rows = h[1];
    // (exact candidate pairs: the cursor counts the candidates staged, the
    // chunk totals the rows kept)
    if (c->ref_pairs_pass ? h[0] < h[1] : h[0] != h[1])
        return fail(WLD_E_HIP, "internal: staging cursor %llu vs chunk total %llu", h[0], h[1]);
    int order_end = c->gather_cap ? 5 : c->ev_end;  // with no rows (and no gather enqueued) it ends at the scan
    if (rows && lin_count && rows > c->gather_cap) {  // not gathered behind the scan
        WLD_TRY(ensure_outputs(c, rows));
        launch_gather(order_args(c), ptr<uint32_t>(c->chunk_base), r.lin_begin, lin_count, n, (uint32_t)c->L, rows,
                      nullptr, rows, c->has_map ? ptr<uint32_t>(c->site_map) : nullptr, ptr<uint32_t>(c->out_a),
                      ptr<uint32_t>(c->out_b), ptr<float>(c->out_d), ptr<float>(c->out_dp), ptr<float>(c->out_r2),
                      c->stream);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(c->ev[5], c->stream));
        HIP_TRY(hipEventSynchronize(c->ev[5]));
        WLD_TRY(check_guard(c, "reference-order gather"));
        order_end = 5;
    }
    c->rows = rows;
    c->have_rows = true;
    c->spec_gather = rows > 0;
    c->gather_cap = 0;
    c->stats.kernel = c->kernel;
    c->stats.pairs = r.pairs;
    c->stats.rows = rows;
    c->times_pending = true;  // (pair_kernel_ms, order_ms, screen_ms: materialize_times)
    c->times_order_end = order_end;
    // (exact candidate pairs: the i8 pass, ref_sums_kernel, ref_compact_kernel)
    c->stats.pair_kernel_launches = c->n_tiles ? (c->ref_pairs_pass ? 3 : c->screened ? 2 : 1) : 0;
    c->stats.tiles = c->n_tiles;
    c->stats.screened = c->ref_pairs_pass ? 4 : c->screened ? (c->screened2 ? 3 : 1) : 0;
    c->stats.screen_fp6 = c->fp6_pass ? 1 : abandoned ? 2 : 0;
    c->stats.fp6_sampled = c->fp6_sampled ? 1 : 0;
    c->stats.candidate_pairs = c->ref_pairs_pass ? h[0] : 0;
    // auto: a threshold at which even the i8 screen leaves more than half the
    // tiles is not screened from now on (nor any lower one): the screen costs a
    // third of the full three-plane kernel, the candidates as much again; in
    // lib.rs's order the exact candidate pairs take over there (a screened
    // tile with one uncertain 16x16 sub-block costs ~0.12 us on the f32
    // kernel: half the C4 tiles ~3 ms over the 0.9 ms screen, about the exact
    // candidate pairs' cost)
    // ... and one at which the two-plane screen (0.8 of the full kernel's
    // time at BASELINE config 4, archive/profiles_r01_r03/r02s2/) leaves more than a fifth
    // goes to the full kernel (the exact mode; lib.rs's order takes the two-
    // plane screen only when asked, WLD_OPT_SCREEN 3)
    // ... the fp6 screen first hands over to the i8 one (a tighter bound at
    // twice the cost) once it leaves more than a sixteenth of the tiles (or,
    // in auto, gives the pass up on reaching that many: the loop above)
    if (c->fp6_pass && h[2] * 16 > c->n_tiles) {
        c->fp6_bad_thr = std::max(c->fp6_bad_thr, r.thr);
    } else if (c->screened && !c->ref_pairs_pass && !c->screened2 && h[2] * 2 > c->n_tiles) {
        c->screen_bad_thr = std::max(c->screen_bad_thr, r.thr);
    }
    if (c->screened && c->screened2 && h[2] * 5 > c->n_tiles) c->screen2_bad_thr = std::max(c->screen2_bad_thr, r.thr);
    // exact candidate pairs, each summed alone in lib.rs's order (~1 ms per
    // million at C4 size): past a tenth of all pairs the full f32 kernel
    // (27.8 ms for every tile at C4) is cheaper
    if (c->ref_pairs_pass && h[0] * 10 > r.pairs) c->ref_pairs_bad_thr = std::max(c->ref_pairs_bad_thr, r.thr);
    c->times_screened = c->screened;
    c->stats.candidate_tiles = c->screened ? h[2] : c->n_tiles;
    c->stats.candidate_blocks = c->screened && !c->ref_pairs_pass ? h[3] : 16 * (uint64_t)c->n_tiles;
    if (n_rows) *n_rows = rows;
    return WLD_OK;
}

int run_chunks(wld_ctx *c, float thr, uint32_t lin_begin, uint32_t lin_end, uint64_t *n_rows) {
    WLD_TRY(run_enqueue(c, thr, lin_begin, lin_end, nullptr));
    return run_complete(c, n_rows);
}
}  // namespace

int wld_run(wld_ctx *c, float thr, uint32_t rb, uint32_t re, uint64_t *n_rows) {
    WLD_TRY(set_dev(c));
    if (!c->loaded) return fail(WLD_E_STATE, "wld_run before wld_load");
    const uint32_t n = chunk_rows_of(c->L);
    if (re == 0 || re > n) re = n;
    if (rb > re) return fail(WLD_E_ARG, "row range [%u,%u) invalid", rb, re);
    uint32_t lb, le;
    rows_to_linear(n, rb, re, lb, le);
    return run_chunks(c, thr, lb, le, n_rows);
}

int wld_run_chunks(wld_ctx *c, float thr, uint32_t chunk_begin, uint32_t chunk_end, uint64_t *n_rows) {
    WLD_TRY(set_dev(c));
    if (!c->loaded) return fail(WLD_E_STATE, "wld_run_chunks before wld_load");
    const uint32_t m = chunks_of(c->L);
    if (chunk_end == 0 || chunk_end > m) chunk_end = m;
    if (chunk_begin > chunk_end) return fail(WLD_E_ARG, "chunk range [%u,%u) invalid", chunk_begin, chunk_end);
    return run_chunks(c, thr, chunk_begin, chunk_end, n_rows);
}

int wld_run_chunks_async(wld_ctx *c, float thr, uint32_t chunk_begin, uint32_t chunk_end, void *d_count_out) {
    WLD_TRY(set_dev(c));
    if (!c->loaded) return fail(WLD_E_STATE, "wld_run_chunks_async before wld_load");
    const uint32_t m = chunks_of(c->L);
    if (chunk_end == 0 || chunk_end > m) chunk_end = m;
    if (chunk_begin > chunk_end) return fail(WLD_E_ARG, "chunk range [%u,%u) invalid", chunk_begin, chunk_end);
    return run_enqueue(c, thr, chunk_begin, chunk_end, static_cast<unsigned long long *>(d_count_out));
}

int wld_run_wait(wld_ctx *c, uint64_t *n_rows) {
    WLD_TRY(set_dev(c));
    return run_complete(c, n_rows);
}

int wld_run_after(wld_ctx *c, wld_ctx *prev) {
    if (!c || !prev) return fail(WLD_E_ARG, "null context");
    if (!c->members.empty() || !prev->members.empty()) return fail(WLD_E_ARG, "wld_run_after on a device group");
    if (c->pend.active) return fail(WLD_E_STATE, "wld_run_after during a run of ctx");
    if (!prev->pend.active) return WLD_OK;  // nothing in flight
    WLD_TRY(set_dev(c));
    // ev[6] separates a screened pass's screen from its candidate launch;
    // ev[3] follows the pair kernel(s) (enqueue_pass)
    if (c->stream == prev->stream) return WLD_OK;  // one stream: already in order
    HIP_TRY(hipStreamWaitEvent(c->stream, prev->screened ? prev->ev[6] : prev->ev[3], 0));
    return WLD_OK;
}

int wld_set_stream(wld_ctx *c, void *stream) {
    if (!c) return fail(WLD_E_ARG, "null context");
    if (!c->members.empty()) return fail(WLD_E_ARG, "wld_set_stream on a device group");
    if (c->pend.active) return fail(WLD_E_STATE, "wld_set_stream during a run");
    WLD_TRY(set_dev(c));
    HIP_TRY(hipStreamSynchronize(c->stream));  // work already queued completes first
    c->stream = stream ? static_cast<hipStream_t>(stream) : c->own_stream;
    return WLD_OK;
}

void *wld_stream(wld_ctx *c) { return c ? (void *)c->stream : nullptr; }

int wld_rows_device(wld_ctx *c, wld_pairs *v) {
    if (!c || !v) return fail(WLD_E_ARG, "null argument");
    if (!c->have_rows) return fail(WLD_E_STATE, "no rows: call wld_run first");
    v->n = c->rows;
    v->site_a = ptr<uint32_t>(c->out_a);
    v->site_b = ptr<uint32_t>(c->out_b);
    v->d = ptr<float>(c->out_d);
    v->d_prime = ptr<float>(c->out_dp);
    v->r2 = ptr<float>(c->out_r2);
    return WLD_OK;
}

int wld_rows_copy(wld_ctx *c, uint32_t *site_a, uint32_t *site_b, float *d, float *d_prime, float *r2) {
    WLD_TRY(set_dev(c));
    if (!c->have_rows) return fail(WLD_E_STATE, "no rows: call wld_run first");
    const size_t n = c->rows;
    if (n) {
        if (site_a) HIP_TRY(hipMemcpyAsync(site_a, c->out_a.p, n * 4, hipMemcpyDeviceToHost, c->stream));
        if (site_b) HIP_TRY(hipMemcpyAsync(site_b, c->out_b.p, n * 4, hipMemcpyDeviceToHost, c->stream));
        if (d) HIP_TRY(hipMemcpyAsync(d, c->out_d.p, n * 4, hipMemcpyDeviceToHost, c->stream));
        if (d_prime) HIP_TRY(hipMemcpyAsync(d_prime, c->out_dp.p, n * 4, hipMemcpyDeviceToHost, c->stream));
        if (r2) HIP_TRY(hipMemcpyAsync(r2, c->out_r2.p, n * 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    return WLD_OK;
}

int wld_rows_copy_device(wld_ctx *c, void *site_a, void *site_b, void *d, void *d_prime, void *r2) {
    WLD_TRY(set_dev(c));
    if (!c->have_rows) return fail(WLD_E_STATE, "no rows: call wld_run first");
    const size_t n = c->rows;
    if (n) {
        if (site_a) HIP_TRY(hipMemcpyAsync(site_a, c->out_a.p, n * 4, hipMemcpyDeviceToDevice, c->stream));
        if (site_b) HIP_TRY(hipMemcpyAsync(site_b, c->out_b.p, n * 4, hipMemcpyDeviceToDevice, c->stream));
        if (d) HIP_TRY(hipMemcpyAsync(d, c->out_d.p, n * 4, hipMemcpyDeviceToDevice, c->stream));
        if (d_prime) HIP_TRY(hipMemcpyAsync(d_prime, c->out_dp.p, n * 4, hipMemcpyDeviceToDevice, c->stream));
        if (r2) HIP_TRY(hipMemcpyAsync(r2, c->out_r2.p, n * 4, hipMemcpyDeviceToDevice, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    return WLD_OK;
}

int wld_dense(wld_ctx *c, float *d, float *d_prime, float *r2, uint8_t *valid) {
    WLD_TRY(set_dev(c));
    if (!c->loaded) return fail(WLD_E_STATE, "wld_dense before wld_load");
    if (!d || !d_prime || !r2 || !valid) return fail(WLD_E_ARG, "wld_dense: null output");
    const size_t L = c->L, LL = L * L;
    if (LL == 0) return WLD_OK;
    if (L > 8192) return fail(WLD_E_ARG, "wld_dense is for tests (n_sites <= 8192)");
    WLD_TRY(build_tiles(c, 0, chunks_of(L)));
    DevBuf dd, ddp, dr2, dv;
    int st = WLD_OK;
    if ((st = ensure(dd, LL * 4)) || (st = ensure(ddp, LL * 4)) || (st = ensure(dr2, LL * 4)) || (st = ensure(dv, LL))) {
        release(dd); release(ddp); release(dr2); release(dv);
        return st;
    }
    DenseArgs da{ptr<float>(dd), ptr<float>(ddp), ptr<float>(dr2), ptr<uint8_t>(dv)};
    (void)hipMemsetAsync(dv.p, 0, LL, c->stream);
    OrderArgs o = order_args(c);
    st = launch_pairs(c, 0.0f, o, &da);
    if (st == WLD_OK) {
        hipError_t e = hipSuccess;
        if (e == hipSuccess) e = hipMemcpyAsync(d, dd.p, LL * 4, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(d_prime, ddp.p, LL * 4, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(r2, dr2.p, LL * 4, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(valid, dv.p, LL, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) st = fail(WLD_E_HIP, "wld_dense copy: %s", hipGetErrorString(e));
    }
    release(dd); release(ddp); release(dr2); release(dv);
    return st;
}

int wld_last_stats(wld_ctx *c, wld_run_stats *out) {
    if (!c || !out) return fail(WLD_E_ARG, "null argument");
    if (c->members.empty()) {
        (void)hipSetDevice(c->device);
        materialize_times(c);
    }
    *out = c->stats;
    return WLD_OK;
}

void wld_pairs_free(wld_pairs *p) {
    if (!p) return;
    free(p->site_a);
    free(p->site_b);
    free(p->d);
    free(p->d_prime);
    free(p->r2);
    memset(p, 0, sizeof(*p));
}

namespace {
// The chunks [lb, le) of the loaded set, rows to host: batches of whole
// chunks, contiguous in the reference order, of at most opt_host_batch_pairs
// (2^31) pairs each (a run's staging positions are 32-bit); their rows
// concatenate in order.  on_chunk (may be null) gets each chunk's pair count
// as the chunk completes, on the calling thread.
int run_host_range(wld_ctx *c, float r2_threshold, uint32_t lb, uint32_t le,
                   const std::function<void(uint64_t)> *on_chunk, wld_pairs *out) {
    memset(out, 0, sizeof(*out));
    WLD_TRY(set_dev(c));
    if (!c->loaded) return fail(WLD_E_STATE, "wld_run_host before wld_load");
    c->stats.progress_filled = 0;
    const uint64_t limit = std::max<uint64_t>(1, c->opt_host_batch_pairs);
    uint64_t cap = 0, done = 0, pairs_done = 0;
    auto grow = [&](uint64_t need) -> int {
        if (need <= cap) return WLD_OK;
        uint64_t k = std::max<uint64_t>(need, cap + cap / 2);
        void *p[5] = {realloc(out->site_a, k * 4), nullptr, nullptr, nullptr, nullptr};
        if (p[0]) out->site_a = (uint32_t *)p[0];
        if (p[0] && (p[1] = realloc(out->site_b, k * 4))) out->site_b = (uint32_t *)p[1];
        if (p[1] && (p[2] = realloc(out->d, k * 4))) out->d = (float *)p[2];
        if (p[2] && (p[3] = realloc(out->d_prime, k * 4))) out->d_prime = (float *)p[3];
        if (p[3] && (p[4] = realloc(out->r2, k * 4))) out->r2 = (float *)p[4];
        if (!p[4]) return fail(WLD_E_OOM, "host allocation of %llu rows failed", (unsigned long long)k);
        cap = k;
        return WLD_OK;
    };
    int st = grow(1);
    for (uint32_t b = lb; st == WLD_OK && b < le;) {
        uint32_t e = b;
        uint64_t pairs = 0;
        while (e < le) {
            const uint64_t p1 = pairs_in_chunks(c->L, e, e + 1);
            if (e > b && pairs + p1 > limit) break;
            pairs += p1;
            ++e;
        }
        uint64_t rows = 0;
        c->on_chunk = on_chunk;
        st = run_chunks(c, r2_threshold, b, e, &rows);
        c->on_chunk = nullptr;
        if (st != WLD_OK) break;
        if ((st = grow(done + rows)) != WLD_OK) break;
        if (rows &&
            (st = wld_rows_copy(c, out->site_a + done, out->site_b + done, out->d + done, out->d_prime + done,
                                out->r2 + done)) != WLD_OK)
            break;
        done += rows;
        pairs_done += pairs;
        b = e;
    }
    if (st != WLD_OK) {
        wld_pairs_free(out);
        return st;
    }
    out->n = done;
    c->stats.pairs = pairs_done;
    c->stats.rows = done;
    return WLD_OK;
}

// wld_run_host on a device group: member k runs shard k of the reference's
// chunk sequence (wld_shard_chunks: contiguous, balanced by pair count) on
// its own host thread (each run blocks on its device); the members' chunk
// completions queue up for the calling thread, which reports them (on_chunk)
// and concatenates the shards' rows in DESCENDING shard order (shard 0 holds
// the last chunks).
int run_host_group(wld_ctx *g, float thr, const std::function<void(uint64_t)> *on_chunk, wld_pairs *out) {
    const int G = (int)g->members.size();
    const size_t L = g->members[0]->L;
    std::vector<wld_pairs> part(G);
    std::vector<int> status(G, WLD_OK);
    std::vector<std::string> msg(G);
    std::vector<uint64_t> pairs(G, 0);
    std::mutex mu;
    std::condition_variable cv;
    std::vector<int> finished;
    // every shard's range before any thread starts: an early return must not
    // leave a joinable std::thread behind (std::terminate)
    std::vector<uint32_t> lb(G), le(G);
    for (int k = 0; k < G; ++k) {
        WLD_TRY(wld_shard_chunks(L, G, k, &lb[k], &le[k]));
        pairs[k] = pairs_in_chunks(L, lb[k], le[k]);
    }
    std::deque<uint64_t> events;  // chunk pair counts from the members, in completion order
    const std::function<void(uint64_t)> push = [&](uint64_t p) {
        std::lock_guard<std::mutex> lk(mu);
        events.push_back(p);
        cv.notify_one();
    };
    std::vector<std::thread> th;
    for (int k = 0; k < G; ++k) {
        th.emplace_back([&, k] {
            const int st = run_host_range(g->members[k], thr, lb[k], le[k], on_chunk ? &push : nullptr, &part[k]);
            std::lock_guard<std::mutex> lk(mu);
            status[k] = st;
            if (st != WLD_OK) msg[k] = wld_last_error();
            finished.push_back(k);
            cv.notify_one();
        });
    }
    uint64_t pairs_done = 0;
    for (;;) {  // progress on the calling thread, chunk by chunk
        std::deque<uint64_t> batch;
        bool all_done;
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return !events.empty() || (int)finished.size() == G; });
            batch.swap(events);
            all_done = (int)finished.size() == G;
        }
        for (uint64_t p : batch) (*on_chunk)(p);
        if (all_done) {
            std::lock_guard<std::mutex> lk(mu);
            if (events.empty()) break;
        }
    }
    for (auto &t : th) t.join();
    for (int k = 0; k < G; ++k) pairs_done += pairs[k];
    int st = WLD_OK;
    for (int k = 0; k < G; ++k)
        if (status[k] != WLD_OK && st == WLD_OK) st = fail(status[k], "device %d (shard %d): %s", g->members[k]->device, k, msg[k].c_str());
    uint64_t total = 0;
    for (auto &p : part) total += p.n;
    if (st == WLD_OK) {
        const uint64_t n = std::max<uint64_t>(total, 1);
        out->site_a = (uint32_t *)malloc(n * 4);
        out->site_b = (uint32_t *)malloc(n * 4);
        out->d = (float *)malloc(n * 4);
        out->d_prime = (float *)malloc(n * 4);
        out->r2 = (float *)malloc(n * 4);
        if (!out->site_a || !out->site_b || !out->d || !out->d_prime || !out->r2)
            st = fail(WLD_E_OOM, "host allocation of %llu rows failed", (unsigned long long)total);
    }
    if (st == WLD_OK) {
        uint64_t at = 0;
        for (int k = G - 1; k >= 0; --k) {
            const wld_pairs &p = part[k];
            memcpy(out->site_a + at, p.site_a, p.n * 4);
            memcpy(out->site_b + at, p.site_b, p.n * 4);
            memcpy(out->d + at, p.d, p.n * 4);
            memcpy(out->d_prime + at, p.d_prime, p.n * 4);
            memcpy(out->r2 + at, p.r2, p.n * 4);
            at += p.n;
        }
        out->n = total;
    } else {
        wld_pairs_free(out);
    }
    for (auto &p : part) wld_pairs_free(&p);
    for (wld_ctx *m : g->members) {
        (void)hipSetDevice(m->device);
        materialize_times(m);
    }
    g->stats = g->members[0]->stats;
    g->stats.progress_filled = 0;
    for (wld_ctx *m : g->members) g->stats.progress_filled += m->stats.progress_filled;
    g->stats.pairs = pairs_done;
    g->stats.rows = st == WLD_OK ? total : 0;
    double kms = 0.0;
    for (wld_ctx *m : g->members) kms = std::max(kms, m->stats.pair_kernel_ms);
    g->stats.pair_kernel_ms = kms;  // the slowest device's last batch
    return st;
}

}  // namespace

int wld_run_host(wld_ctx *c, float r2_threshold, wld_progress_fn progress, void *user, wld_pairs *out) {
    if (!out) return fail(WLD_E_ARG, "null out");
    memset(out, 0, sizeof(*out));
    if (!c) return fail(WLD_E_ARG, "null context");
    // lib.rs:670-674: per chunk, the running count of pairs in the chunks
    // completed BEFORE it (fetch_add's previous value)
    uint64_t before = 0;
    const std::function<void(uint64_t)> on_chunk = [&](uint64_t p) {
        progress(before, user);
        before += p;
    };
    const std::function<void(uint64_t)> *oc = progress ? &on_chunk : nullptr;
    if (!c->members.empty()) {
        for (wld_ctx *m : c->members)
            if (!m->loaded) return fail(WLD_E_STATE, "wld_run_host before wld_load");
        return run_host_group(c, r2_threshold, oc, out);
    }
    return run_host_range(c, r2_threshold, 0, chunks_of(c->L), oc, out);
}

int wld_all_weighted_ld_pairs(wld_ctx *c, const uint8_t *sites, size_t n_sites, size_t n_seqs,
                              const uint64_t *site_map, const float *weights, float r2_threshold,
                              wld_progress_fn progress, void *user, wld_pairs *out) {
    if (!out) return fail(WLD_E_ARG, "null out");
    memset(out, 0, sizeof(*out));
    if (progress) progress(0, user);  // lib.rs:584
    WLD_TRY(wld_load(c, sites, n_sites, n_seqs, site_map, weights));
    return wld_run_host(c, r2_threshold, progress, user, out);
}

int wld_single_weighted_ld_pair(wld_ctx *c, const uint8_t *a, const uint8_t *b, const float *weights, size_t n_seqs,
                                float out[3]) {
    if (!a || !b || !weights || !out) return fail(WLD_E_ARG, "null argument");
    if (c && !c->members.empty()) {
        // one pair: the first device; the group's loaded set is replaced (as
        // on a single context), so every member needs a new wld_load
        for (wld_ctx *m : c->members) m->loaded = false;
        c = c->members[0];
    }
    std::vector<uint8_t> buf(2 * n_seqs);
    memcpy(buf.data(), a, n_seqs);
    memcpy(buf.data() + n_seqs, b, n_seqs);
    WLD_TRY(wld_load(c, buf.data(), 2, n_seqs, nullptr, weights));
    float d[4], dp[4], r2[4];
    uint8_t v[4];
    WLD_TRY(wld_dense(c, d, dp, r2, v));
    if (!v[1]) return 0;
    out[0] = d[1];
    out[1] = dp[1];
    out[2] = r2[1];
    return 1;
}

}  // extern "C"
