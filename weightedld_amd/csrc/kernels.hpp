// Device-side layout and launchers shared by capi.hip and the kernel files.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace wld {

// ---- layout constants (see DESIGN.md "Data layout in HBM") ----
constexpr int kChunk = 256;      // reference chunk side, lib.rs:615
constexpr int kTile = 64;        // pair-kernel tile side (sites); 4 tiles per chunk side
constexpr int kSeqPad = 64;      // sequences padded to a multiple of this
constexpr int kTilesPerChunk = kChunk / kTile;
// an empty slot of a reordered tile list (never a real tile: T_used < 65535 there)
constexpr uint32_t kNoTile = 0xFFFFFFFFu;

// Code byte per (site, sequence): bit0 = sequence is major or minor at the site
// ("in" the pair mask, lib.rs:435), bit1 = sequence is major (lib.rs:430,432).
constexpr uint8_t kCodeIn = 1;
constexpr uint8_t kCodeMaj = 2;

struct OrderArgs {
    // staging written by the pair kernels (filtered indices, unordered tiles)
    uint32_t *st_a, *st_b;
    float *st_d, *st_dp, *st_r2;
    uint64_t st_capacity;
    // per (site a, 64-wide b tile) segment: count (<= 64) and staging offset
    uint8_t *seg_cnt;   // [LP][T]
    uint32_t *seg_off;  // [LP][T]
    uint32_t T;         // number of 64-wide tiles (LP / 64)
    uint32_t *chunk_total;  // [n_chunks_total] rows per reference chunk (linear triu index)
    unsigned long long *cursor;  // staging allocation cursor
    // per-chunk progress (lib.rs:670-674; wld_run_host with a callback, else
    // null): tiles left per linear chunk; the workgroup that finishes a
    // chunk's last tile appends the chunk's pair count to the mapped host log
    // at slot atomicAdd(prog_n, 1) (tile_done, pair_common.hpp)
    unsigned *chunk_left;
    unsigned *prog_n;
    unsigned long long *prog_log;
    uint32_t L;  // sites of the loaded set (a chunk's pair count)
    // guard word in mapped host memory (report_guard): a kernel that finds an
    // index out of range (a candidate-list entry, a tile, a staged pair, a
    // gather destination) records what it found here and skips the access
    // instead of faulting the context; run_complete turns it into WLD_E_STATE
    unsigned *guard;
};

// report_guard bits (wld_run_stats.guard and the WLD_E_STATE message)
enum : unsigned {
    kGuardEntry = 1u,   // a candidate-list entry outside the list's buckets
    kGuardTile = 2u,    // a listed tile with ta > tb or tb past the set's last tile
    kGuardPair = 4u,    // a staged candidate pair with a >= b or b past the set
    kGuardSlice = 8u,   // a candidate slice outside staging or with a bad tile
    kGuardGather = 16u  // a gather destination past the run's row count, or a source past staging
};
__device__ inline void report_guard(const OrderArgs &o, unsigned bit) {
    if (o.guard) __hip_atomic_store(o.guard, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// a tile (ta << 16 | tb) the pair kernels may compute: ta <= tb < T_used
__device__ inline bool tile_in_range(uint32_t tile, uint32_t L) {
    const uint32_t ta = tile >> 16, tb = tile & 0xFFFFu;
    return ta <= tb && (uint64_t)tb * kTile < L;
}

// The run's chunk scan (order.hip): exclusive scan of the chunk totals
// [lin_begin, lin_begin + count) into chunk_base; the row total into *total,
// *count_out (may be null) and host_out[1], the staging cursor into
// host_out[0], the candidate-tile count cand_count[0] into host_out[2] and
// their computed 16x16 sub-blocks cand_count[1] into host_out[3] (host_out:
// mapped pinned memory, may be null); cursor, the chunk totals and both
// candidate counts are left at 0 for the next run.  With ticket set, the last
// workgroup of the candidate launch after a screen runs it (scan_tail,
// pair_common.hpp) instead of a launch of its own.
struct ScanArgs {
    uint32_t *chunk_total;
    uint32_t lin_begin, count;
    uint32_t *chunk_base;
    unsigned long long *total, *cursor, *host_out, *count_out;
    unsigned long long *cursor_seen;  // device word: the staging cursor before its reset (may be null)
    unsigned *cand_count;  // this pass's {candidate tiles, their candidate sub-blocks} (read)
    // the OTHER candidate set (the next pass's: {count, sub-blocks} and 16
    // bucket counts), zeroed here; this pass's set is never written by its
    // own scan, so a workgroup still reading it cannot see it reset (capi.hip
    // enqueue_pass alternates the sets by pass parity)
    unsigned *cand_reset;
    unsigned *cand_buckets_reset;
    unsigned *ticket;  // 0 between launches; null: the scan is launched on its own
};

// 64-bit words of a context's run counters (capi.hip enqueue_pass):
// {cursor, total, {ticket, work}, set 0: {candidates, sub-blocks} + 16 bucket
// counts (9 words), set 1: the same, the cursor the scan saw}
constexpr uint32_t kCounterWords = 22;
constexpr uint32_t kCursorSeen = 21;
// set on a pass's candidate count and on its bucket 0 by a screen that gave
// up (the fp6 screen past ScreenArgs::bail candidates): the candidate launch
// then computes nothing, the scan reports the count with the bit to the host
// (which re-runs the pass on the i8 screen) and a cursor the gather enqueued
// behind it refuses
constexpr unsigned kAbandonBit = 0x80000000u;
constexpr uint32_t kCandSetWords = 9;
constexpr uint32_t kCandSet0 = 3;

struct DenseArgs {
    float *d, *dp, *r2;
    uint8_t *valid;
};

// encode.hip
// site_index: nullptr, or the kept-site map of the device pre-pass (row s of the
// filtered set = raw row site_index[s])
void launch_encode(const uint8_t *d_sites, const uint32_t *site_index, size_t L, size_t N, size_t LP, size_t NP,
                   uint8_t *codes, uint8_t *site_ok, hipStream_t s);
void launch_weight_prep(const float *d_w, size_t N, size_t NP, float *w_pad, float *wstats, hipStream_t s);

// prepass.hip (device site filter + Henikoff weights, bit-exact with host.cpp)
void launch_site_stats(const uint8_t *raw, size_t L, size_t N, uint32_t min_acgt, float min_minor, float max_minor,
                       uint8_t *keep, float *tab, hipStream_t s);
void launch_henikoff(const uint8_t *raw, const uint32_t *site_index, size_t n_kept, size_t N, const float *tab,
                     float *tabK, float *w, hipStream_t s);
void launch_fill_ones(float *w, size_t N, hipStream_t s);

// pair_valu.hip
struct ValuLaunch {
    const uint8_t *codes;    // site-major codes, NP bytes per site (REF: the lane-class layout)
    const float *w;          // NP weights (REF: the lane-class layout)
    const uint8_t *site_ok;
    const uint32_t *tiles;   // tile list (or the candidate list with tile_count)
    uint32_t n_tiles;        // list length, or (tile_count) its capacity
    const unsigned *tile_count;  // device tile count: the looping candidate launch; else null
    uint32_t L, NP, n_chunk_rows;
    float thr;
    bool safe;   // non-finite weights: the select loop
    bool plain;  // WLD_OPT_VALU_PLAIN: the VALU fmaf loop instead of f32 MFMA
    bool ref;    // WLD_OPT_REF_SUMS: lib.rs's own f32 summation order
    uint32_t ref_cls;  // REF: sequence positions per lane class (multiple of 64, 0 when N < 8)
    uint32_t ref_tail_n;  // REF: the scalar tail's sequences (N mod 8), in the stage after the classes
    // tile_count launches: per list entry, the 16x16 sub-blocks (bit 4 (a/16)
    // + b/16) whose pairs are computed; the others' pairs provably fail (the
    // screen's per-pair bound) and are skipped.  Null: every sub-block.
    const uint32_t *tile_bits;
    unsigned *tile_work;  // tile_count launches: the work counter (0 before the launch)
    // tile_count launches: the list in 16 buckets of bucket_cap entries
    // (pair_common.hpp cand_entry; null: one plain list)
    const unsigned *tile_buckets;
    uint32_t bucket_cap;
    ScanArgs scan;        // tile_count launches: the run's scan fused into the last workgroup (ticket set)
    // tile_count launches: the list's entries are 16-row blocks of candidate
    // tiles (pair_mfma.hip ScreenArgs::rb_items), counted by the buckets
    bool rb_items;
};
// returns true when the run's chunk scan ran in the launch (v.scan given, the
// item kernel of a full run); else the caller launches it
bool launch_pair_valu(const ValuLaunch &v, const OrderArgs &o, const DenseArgs *dense, hipStream_t s);
// The candidate pairs a kModeRefPairs launch (pair_mfma.hip) staged: summed in
// lib.rs's order one pair per thread from the lane-class layout
// (ref_sums_kernel), then per tile slice the passing rows kept in place (in
// order), its segment counts/offsets and chunk total corrected, the rest
// dropped (ref_compact_kernel, whose last workgroup runs the run's chunk scan:
// scan.ticket).
struct RefRowsLaunch {
    const uint8_t *rcodes;  // the lane-class layout (NPr bytes per site)
    const float *rw;
    uint32_t NPr, ref_cls, ref_tail_n, n_chunk_rows;
    float thr;
    const uint32_t *slices;  // per tile with candidates: {staging base, rows, ta << 16 | tb}
    const unsigned *slice_count;
    unsigned *work;  // work counter, 0 before the launch
    ScanArgs scan;
};
void launch_ref_rows(const RefRowsLaunch &r, const OrderArgs &o, hipStream_t s);
// the lane-class layout of REF: cls positions per class, the tail stage, NPr
void ref_layout_dims(size_t N, uint32_t *cls, uint32_t *tail, size_t *NPr);
void launch_ref_layout(const uint8_t *codes, const float *w_pad, size_t LP, size_t NP, size_t N, uint8_t *rcodes,
                       float *rw, hipStream_t s);

// pair_mfma.hip
bool mfma_supported();
// weight digits (two layouts) + per-64-site filter bits
size_t mfma_planes_bytes(size_t LP, size_t NP);
void launch_mfma_prep(const uint8_t *site_ok, const float *w_pad, size_t L, size_t LP, size_t NP, int shift,
                      int8_t *planes, hipStream_t s);
// frag holds 2 LP NP bytes: selector-coded, then 0/1/2-coded (B operands)
void launch_frag(const uint8_t *codes, size_t LP, size_t NP, uint8_t *frag, hipStream_t s);
// weight-plane statistics written by launch_mfma_prep (read back once per load)
struct MfmaWeightStats {
    unsigned plane_mask;  // bit p = digit plane p (of 4) has a nonzero digit
    int nonneg;           // every weight >= 0
    uint64_t resid[3];    // resid[t-1] = sum_k |q_k - 2^(8t) d_t,k|: what top plane t alone leaves out
    uint64_t dsum[4];     // dsum[p] = sum_k |d_p,k|: bounds every one-plane sum of plane p
};
// synchronises s; returns 0, or -1 on a HIP error
int mfma_weight_stats(const int8_t *wplanes, size_t LP, size_t NP, hipStream_t s, MfmaWeightStats *out);

// workgroups of the candidate launch after a screen (it strides over a tile
// list whose length is known only on the device): 4 rounds of 2 per CU
constexpr uint32_t kCandidateGrid = 2048;
// ... and of the reference-order f32 kernel's candidate loop: its resident
// workgroups (three per CU, 256 CUs); extra workgroups would only queue (and
// cost dispatch time when there is no candidate at all)
constexpr uint32_t kRefCandidateGrid = 768;
// ... and of its items (ref_item_kernel<LOOP>, one sub-block per wave, five
// workgroups per CU): 1,024 (4 per CU) measured faster than 768, 896 or
// every slot (1,280) on LD blocks (profiles/r06t/, r06u/)
constexpr uint32_t kRefItemGrid = 1024;
// ... and of ref_sums_kernel / ref_compact_kernel (low-register: eight per CU)
constexpr uint32_t kRefRowsGrid = 2048;

// The fp6 screen's operands (pair_mfma.hip frag6_kernel) and constants: R
// (residual bound of the rounded weights plus the reference's rounding) and
// Tg (>= every doubled T), in the units of the fp6 weights (capi.hip).
struct Fp6Screen {
    const uint8_t *a6, *b6;
    uint32_t NK;  // 128-sequence blocks
    double R;
    float Tg;
};
size_t fp6_a_bytes(size_t LP, size_t NP);
size_t fp6_b_bytes(size_t LP, size_t NP);
// w6: NP fp6 (e2m3) codes of the rounded weights (0 for padding)
void launch_frag6(const uint8_t *codes, const uint8_t *w6, size_t LP, size_t NP, uint8_t *a6, uint8_t *b6,
                  hipStream_t s);

// The i8 one-plane screen's pre-multiplied operand images (pair_mfma.hip
// pair_i8_screen2w_kernel; capi.hip i8img_prepare): A = the top weight digit
// times in / major, B = the codes, per 64-site tile and 64-sequence block.
struct I8Screen {
    const uint8_t *a8, *b8;
    uint32_t digit_plane;  // the digit plane the images hold
};
size_t i8_a_bytes(size_t LP, size_t NP);
size_t i8_b_bytes(size_t LP, size_t NP);
// digit: NP int8 digits of the plane (planes + plane * NP)
void launch_i8img(const uint8_t *codes, const int8_t *digit, size_t LP, size_t NP, uint8_t *a8, uint8_t *b8,
                  hipStream_t s);

struct MfmaLaunch {
    const uint8_t *codes;   // site-major codes (used when frag is null)
    const uint8_t *frag;    // fragment-major selector-coded copy (LDS kernel), or null
    const uint8_t *frag_b;  // fragment-major 0/1/2-coded copy (B operands)
    const int8_t *wplanes;
    const uint32_t *tiles;
    uint32_t n_tiles, L, LP, NP, n_chunk_rows;
    float thr;
    int shift;
    unsigned plane_mask;
    int nonneg;
    bool prefilter;  // thr > 0: skip pairs r2_bound_skip rejects
    bool screen;     // with the prefilter: one-plane screen, then candidates
    bool screen2;    // the screen on the top two digit planes (>= 3 active planes)
    uint64_t resid[3];
    uint64_t dsum[4];
    uint32_t *cand_list;   // 32 n_tiles entries: 16 buckets of tiles, then 16 of their sub-block bits
    unsigned *cand_count;  // 0 before the launch (chunk_scan_kernel resets it)
    unsigned *cand_buckets;  // 16 bucket counts, 0 before the launch (chunk_scan_kernel resets them)
    int test_guard = 0;      // WLD_OPT_TEST_GUARD (launch_candidates)
    unsigned *cand_work;   // the candidate launch's work counter (the screen zeroes it)
    // WLD_OPT_REF_SUMS: the candidate tiles go to the reference-order f32
    // kernel (ref_valu, tiles/tile_count filled in here) and the screen's
    // residual bound grows by r_extra_q (fixed-point units: how far the
    // reference's f32 sums can lie from the fixed-point sums, 2x2-cell L1)
    const ValuLaunch *ref_valu;
    double r_extra_q;
    // WLD_OPT_REF_SUMS without a screen: every tile on all planes, the pairs
    // the bound cannot reject (residual r_extra_q) staged as candidates, then
    // summed one by one in lib.rs's order (launch_ref_rows; ref_rows filled in
    // here but for the slices, count and work counter)
    const RefRowsLaunch *ref_rows;
    // with a screen: the run's scan, fused into the screen's or the candidate
    // launch's last workgroup when scan.ticket is set
    ScanArgs scan;
    // the one-plane screen on fp6 x fp4 MFMA instead of i8 (null: the i8 screen)
    const Fp6Screen *fp6;
    // ... gives up past this many candidate tiles (0: never; kAbandonBit)
    uint32_t fp6_bail;
    // ... its tile-pair list (pair_fp6_screen2w_kernel; XCD-ordered, kNoTile padded)
    const uint32_t *f6_pairs;
    uint32_t f6_n_pairs;
    // the i8 one-plane screen on the tile-pair list with pre-multiplied
    // operands (null: the per-tile LDS kernel)
    const I8Screen *i8img = nullptr;
};
// The fp6 screen's sample run over every stride-th entry of its list: probe[0]
// = the sampled tiles holding a pair its bound cannot reject, probe[1] = the
// sampled tiles (m as for the pass; nothing else is written)
void launch_fp6_probe(const MfmaLaunch &m, unsigned *probe, uint32_t stride, hipStream_t s);
// Enqueues the MFMA pair kernel(s) of one pass; returns true when a screen
// (one- or two-plane) ran (then screen_done, if given, is recorded between
// the two launches).
bool launch_pair_mfma(const MfmaLaunch &m, const OrderArgs &o, const DenseArgs *dense, hipStream_t s,
                      hipEvent_t screen_done);

// order.hip
// per-chunk progress of the chunks [lin_begin, lin_begin + count): tiles per
// chunk into chunk_left[lin], prog_n = 0
void launch_progress_init(unsigned *chunk_left, uint32_t lin_begin, uint32_t count, uint32_t n_chunk_rows, uint32_t L,
                          unsigned *prog_n, hipStream_t s);
// zeroes the run state (staging cursor, row total, every chunk total)
void launch_run_init(unsigned long long *counters, uint32_t *chunk_total, uint32_t n_chunks, hipStream_t s);
// the run's chunk scan as a launch of its own (ScanArgs; ticket unused)
void launch_chunk_scan(const ScanArgs &a, hipStream_t s);
// (rows: the run's row count, the bound of every destination.  With state
// (the run counters) set, the gather is enqueued before the host has seen the
// scan: it reads the row total and the cursor the scan saw from the device and
// writes nothing if the staging overflowed or the rows exceed out_cap — the
// host then re-runs the pass or gathers again into larger buffers)
void launch_gather(const OrderArgs &o, const uint32_t *chunk_base, uint32_t lin_begin, uint32_t count,
                   uint32_t n_chunk_rows, uint32_t L, uint64_t rows, const unsigned long long *state,
                   uint64_t out_cap, const uint32_t *site_map, uint32_t *out_a, uint32_t *out_b, float *out_d,
                   float *out_dp, float *out_r2, hipStream_t s);

// Linear index of chunk (row, col) in the reference's triu_index order
// (lib.rs:623-632): rows descend, so row r starts at (n-1-r)(n-r)/2.
__host__ __device__ inline uint32_t chunk_linear(uint32_t n, uint32_t row, uint32_t col) {
    uint32_t rf = n - 1 - row;
    return rf * (rf + 1) / 2 + (col - row);
}

// pairs (a < b) of chunk (row, col) of an L-site set: lib.rs:636-667's loops
__host__ __device__ inline uint64_t chunk_pairs(uint32_t L, uint32_t row, uint32_t col) {
    const uint64_t lo_a = (uint64_t)row * kChunk, lo_b = (uint64_t)col * kChunk;
    const uint64_t ra = lo_a >= L ? 0 : (L - lo_a < (uint64_t)kChunk ? L - lo_a : (uint64_t)kChunk);
    const uint64_t rb = lo_b >= L ? 0 : (L - lo_b < (uint64_t)kChunk ? L - lo_b : (uint64_t)kChunk);
    return row == col ? ra * (ra ? ra - 1 : 0) / 2 : ra * rb;
}

}  // namespace wld
