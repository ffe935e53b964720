/*
 * weightedld.h — C ABI of the MI355X-native WeightedLD all-pairs LD hot path.
 *
 * The reference (ojcharles/WeightedLD, Rust crate rust/weighted_ld) has no FFI;
 * its hot path is the generic Rust fn
 *     pub fn all_weighted_ld_pairs(site_set: &SiteSet, weights: &[f32],
 *                                  r2_threshold: f32,
 *                                  progress_report: impl FnMut(usize) + Send)
 *         -> PairStore<LdStats>                               (lib.rs:578-684)
 * called once from main.rs:180-190.  The entry points below are what a Rust
 * `extern "C"` binding of that seam needs: plain pointers
 * and sizes, no Rust/C++/torch types, no exceptions across the boundary, every
 * call returns a status code (WLD_OK or a negative WLD_E_*), and
 * wld_last_error() gives the message for the calling thread.
 *
 * Symbol codes are the reference's #[repr(u8)] Symbol (lib.rs:20-29):
 *     A=0 C=1 G=2 T=3 Missing('-')=4 Unknown=5
 * A "site-major" buffer is SiteSet.buffer (lib.rs:163): buffer[site*n_seqs+seq].
 */
#ifndef WEIGHTEDLD_H
#define WEIGHTEDLD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ status */
#define WLD_OK 0
#define WLD_E_ARG (-1)    /* bad argument (the reference would panic)           */
#define WLD_E_HIP (-2)    /* HIP runtime error                                   */
#define WLD_E_OOM (-3)    /* device or host allocation failed                    */
#define WLD_E_NODEV (-4)  /* no usable gfx950 device                             */
#define WLD_E_IO (-5)     /* file could not be read / written                    */
#define WLD_E_FORMAT (-6) /* input violates the reference's format (it panics)  */
#define WLD_E_STATE (-7)  /* call order violated (e.g. run before load), or a
                             device guard refused an out-of-range index (the
                             run produced no rows; the context stays usable)    */

#define WLD_SYM_A 0
#define WLD_SYM_C 1
#define WLD_SYM_G 2
#define WLD_SYM_T 3
#define WLD_SYM_MISSING 4
#define WLD_SYM_UNKNOWN 5
#define WLD_NONE (-1) /* Option<Symbol>::None */

const char *wld_status_string(int status);
/* Message of the last failed call on this thread ("" if none). */
const char *wld_last_error(void);
/* Library version string, e.g. "weightedld-amd 0.1.0 (gfx950)". */
const char *wld_version(void);

/* ========================================================================
 * Host pre-pass — stays on the host per north_star.  Mirrors lib.rs:20-380.
 * ======================================================================== */

/* Opaque SiteSet (lib.rs:158-173): site-major symbol buffer, optional
 * site_map (filtered index -> parent index, lib.rs:165-169) and per-site
 * histograms (lib.rs:171-172). */
typedef struct wld_siteset wld_siteset;

/* read_fasta + SiteSet::from_multiseq (lib.rs:277-307, 176-206), including the
 * reader's quirks: every non-'>' line is one sequence and its '\n' becomes a
 * trailing Unknown site.  WLD_E_FORMAT where the reference panics (sequences
 * of unequal length, lib.rs:180-182; no sequence at all, lib.rs:178). */
int wld_read_fasta(const char *path, wld_siteset **out);

/* VCF reader following the Python reference's handle_vcf
 * (WeightedLD.py:311-379): phased diploid calls split into two haplotypes,
 * '.' -> 4 (Missing), allele digits used as symbol codes, the last data line
 * dropped (:365), haplotypes in reversed order (np.rot90, :375) and
 * site_map = POS.  The Rust crate has no VCF input; this serves BASELINE
 * config 3.  WLD_E_FORMAT where the Python code exits. */
int wld_read_vcf(const char *path, wld_siteset **out);

/* Builds a SiteSet from a caller buffer (copied); histograms computed as in
 * from_multiseq (lib.rs:194-196). site_map may be NULL (identity). */
int wld_siteset_from_buffer(const uint8_t *site_major, size_t n_sites, size_t n_seqs,
                            const uint64_t *site_map, wld_siteset **out);
void wld_siteset_free(wld_siteset *s);
size_t wld_siteset_n_sites(const wld_siteset *s);                        /* lib.rs:254-256 */
size_t wld_siteset_n_seqs(const wld_siteset *s);                         /* lib.rs:259-261 */
const uint8_t *wld_siteset_buffer(const wld_siteset *s);                 /* SiteSet.buffer */
const uint64_t *wld_siteset_site_map(const wld_siteset *s);              /* NULL = identity */
uint64_t wld_siteset_parent_site_index(const wld_siteset *s, size_t i);  /* lib.rs:263-265 */
int wld_siteset_histogram(const wld_siteset *s, size_t site, uint64_t out[6]); /* lib.rs:272 */

/* SymbolHistogram::from_slice (lib.rs:98-104) and major_minor_symbols
 * (lib.rs:126-140): ties keep the earlier of A,C,G,T,-; Unknown never
 * eligible; WLD_NONE for None. */
int wld_histogram(const uint8_t *symbols, size_t n, uint64_t out[6]);
int wld_major_minor(const uint64_t hist[6], int *major, int *minor);

/* is_site_of_interest (lib.rs:309-338); min_acgt is the COUNT
 * ceil(min_acgt_frac * n_seqs) of main.rs:139.  Returns 1/0. */
int wld_is_site_of_interest(const uint8_t *site, size_t n, size_t min_acgt, float min_minor,
                            float max_minor);

/* main.rs:139-143: siteset.filter_by(is_site_of_interest) with
 * min_acgt = ceil(min_acgt_frac * n_seqs) (f32 arithmetic), i.e.
 * SiteSet::filter_by (lib.rs:230-251). */
int wld_siteset_filter_sites_of_interest(const wld_siteset *s, float min_acgt_frac,
                                         float min_minor, float max_minor, wld_siteset **out);

/* henikoff_weights (lib.rs:340-380), out has n_seqs floats. */
int wld_henikoff_weights(const wld_siteset *s, float *out);

/* ========================================================================
 * Device hot path — replaces all_weighted_ld_pairs / single_weighted_ld_pair.
 * ======================================================================== */

typedef struct wld_ctx wld_ctx;

/* One context per device; owns its HIP stream, device buffers and results.
 * Not thread-safe; separate contexts are independent.  device = HIP ordinal. */
int wld_create(int device, wld_ctx **out);
/* A context over n_devices devices (HIP ordinals; repeats allowed, e.g. to run
 * several shards on one device in tests): one member context per entry.
 * wld_load replicates the input to every member; wld_run_host and
 * wld_all_weighted_ld_pairs (the reference's one call, lib.rs:578-684, which
 * uses every core) shard the reference's chunk sequence over the members
 * (wld_shard_chunks: contiguous ranges balanced by pair count), run them
 * concurrently, and return the rows in the reference order (shards
 * concatenated in descending shard order).  Options and the kernel choice
 * apply to every member; wld_last_stats reports member 0's kernel with the
 * group's pair/row totals.  Other device entry points fail with WLD_E_STATE
 * on such a context.  With n_devices == 1 it returns a plain single-device
 * context (wld_create(devices[0], out)), on which every entry point works. */
int wld_create_multi(const int *devices, int n_devices, wld_ctx **out);
int wld_n_devices(const wld_ctx *ctx); /* 1, or the member count of a multi-device context */
void wld_destroy(wld_ctx *ctx);

/* Kernel selection.  AUTO (default): the exact-integer MFMA kernel when the
 * weights are finite, their dynamic range fits its fixed-point weight planes
 * (3 digit planes, 23-bit fixed point, when min |w| >= 2^-4 max |w|; 4 planes,
 * 31-bit, when min |w| >= 2^-12 max |w| and n_seqs <= 65,024: every weight
 * within 2^-19 relative) and n_seqs <= 5,592,320 (int32 sums),
 * else the exact-product f32 kernel (WLD_KERNEL_VALU: f32-input MFMA for
 * finite weights, a VALU loop otherwise).  An explicit WLD_KERNEL_MFMA with
 * non-finite or all-zero weights, or more sequences, fails with WLD_E_ARG at
 * load (a wide dynamic range is allowed: small weights lose precision).  Both
 * run on the GPU; there is no CPU path. */
#define WLD_KERNEL_AUTO 0
#define WLD_KERNEL_VALU 1
#define WLD_KERNEL_MFMA 2
int wld_set_kernel(wld_ctx *ctx, int kernel);

/* Per-context options (the library reads no environment variables).  Except
 * WLD_OPT_REF_SUMS none changes a result: every setting gives bit-identical
 * rows; they exist for A/B measurements and tests.  Set between runs; WLD_E_ARG for an unknown
 * option or a bad value.
 *   WLD_OPT_PREFILTER  1 (default): with r2_threshold > 0 the MFMA kernel
 *                      skips the f32 epilogue of pairs that a rigorous bound
 *                      proves cannot pass; 0: every pair.
 *   WLD_OPT_SCREEN     1 (default, auto): with the prefilter on, a screen
 *                      launch on the top nonzero weight-digit plane bounds
 *                      every pair's r2 (the lower planes' share bounded
 *                      exactly; none with a single nonzero plane, e.g. equal
 *                      weights) and only candidate 64x64 tiles are recomputed
 *                      with every plane — unless at this or a higher threshold
 *                      the screen left more than half the tiles as candidates.
 *                      Then (three or more active planes) the screen runs on
 *                      the top two planes, the planes below bounded the same
 *                      way, unless at this or a higher threshold that left more
 *                      than a fifth of the tiles as candidates (then every
 *                      tile goes to the full kernel directly); 2: always the
 *                      one-plane screen; 3: always the two-plane screen (the
 *                      one-plane one with fewer than three active planes);
 *                      0: every tile, every plane.  In lib.rs's order
 *                      (WLD_OPT_REF_SUMS 1) auto replaces the two-plane tier:
 *                      where the one-plane screen does not pay, every tile runs
 *                      once on the top two digit planes, staging the pairs the bound cannot
 *                      reject (the reference's rounding as residual), and only
 *                      those are summed in lib.rs's order, one by one — unless
 *                      at this or a higher threshold they were more than a
 *                      tenth of all pairs (then the full f32 kernel); 4: always
 *                      that path (lib.rs's order; otherwise as 0).
 *   WLD_OPT_TILE_ORDER 0 (default): L2/XCD-aware tile launch order; 1: plain
 *                      (a-tile, b-tile) order.
 *   WLD_OPT_ALL_PLANES 0 (default): all-zero digit planes are skipped; 1: the
 *                      MFMA kernel multiplies all three.
 *   WLD_OPT_MFMA_LAYOUT 0 (default): LDS-streaming fragment-major kernel; 1:
 *                      the site-major register kernel (takes effect at the
 *                      next load).
 *   WLD_OPT_VALU_PLAIN 0 (default): the f32 fallback multiplies on f32-input
 *                      MFMA; 1: a VALU fmaf loop (same sums, same order).
 *   WLD_OPT_REF_SUMS   1 (default): the four masked sums of every pair are
 *                      formed in lib.rs's own f32 order — 8 lane sums of the
 *                      sequences k = j mod 8 (lib.rs:416-445), their ordered
 *                      horizontal sum (packed_simd's x86 f32x8::sum(),
 *                      :447-452), then the scalar tail (:461-480) — on the f32
 *                      kernel, so d, d' and r2 are bit-identical to lib.rs's
 *                      on every input, including pairs whose f32 sums lib.rs
 *                      itself gets wrong (minor alleles carried by a few
 *                      low-weight sequences).  With the MFMA kernel and a
 *                      positive threshold the i8 screen runs first, its bound
 *                      widened by the reference's rounding, and only candidate
 *                      tiles take the f32 kernel.  0: exact sums (integer
 *                      MFMA, all digit planes; the f32 kernel's two-level sums
 *                      when the weights need it) rounded once — more accurate
 *                      than lib.rs, faster where many tiles are candidates
 *                      (linkage, thresholds <= 0), and different from lib.rs
 *                      in the last bits (or more on ill-conditioned pairs).
 *                      The one option that changes results.
 *   WLD_OPT_STAGING_ROWS   initial staging capacity in rows (default 2^25;
 *                      grown on overflow by a re-run).
 *   WLD_OPT_HOST_BATCH_PAIRS  pairs per batch of wld_run_host (default 2^31).
 *   WLD_OPT_SCREEN_FP6 1 (default, auto): the one-plane screen multiplies
 *                      fp6 (e2m3) weights by fp4 codes on the block-scaled
 *                      MFMA (128 sequences per instruction, twice the i8
 *                      rate) when the weights are nonnegative, at most 16,384
 *                      sequences, and their fp6 rounding leaves a residual
 *                      within 2% of the sums or twice the i8 top digit's, at
 *                      thresholds above any at which it left more than a
 *                      quarter of the tiles as candidates; 0: the i8 screen;
 *                      2: fp6 whenever it applies; 3: auto without the
 *                      sample run (below).  Auto decides a threshold it has
 *                      not seen from a sample run first (about 1/64 of the
 *                      tiles screened on fp6, counting only): past a
 *                      sixteenth of them as candidates the pass screens on
 *                      i8.  Same rows (a screen only decides which tiles are
 *                      computed).
 *   WLD_OPT_FUSED_SCAN 1 (default): after a screen, the run's chunk scan runs
 *                      in the candidate launch's last workgroup (ranges up to
 *                      4096 chunks); 0: as a launch of its own (the kernel
 *                      boundary orders it).  Same rows.
 *   WLD_OPT_FP6_PAIRS_MIN_TILES  the fp6 screen computes two tiles of a row
 *                      per workgroup (one shared A operand stream) when the
 *                      run's tile list has at least this many tiles (default
 *                      0: always), else one tile per workgroup.  Same rows.
 *   WLD_OPT_I8_PAIRS   1 (default): the i8 one-plane screen (nonnegative
 *                      weights, at most 16,384 sequences) runs on the fp6
 *                      screen's tile-pair list with wide waves, its operands
 *                      (the top weight digit times the site indicators, and
 *                      the codes) pre-multiplied once per load (3 bytes per
 *                      site and sequence); 0: one tile per workgroup, the
 *                      operands formed per stage.  Same rows.
 *   WLD_OPT_TEST_GUARD 0 (default); 1 (tests only): before each candidate
 *                      launch the last candidate bucket's count is set one
 *                      past its capacity, so the launch meets an entry outside
 *                      the buckets.  Its guard refuses the entry and the run
 *                      fails with WLD_E_STATE instead of reading through it;
 *                      the next run (option back at 0) starts clean.
 *                      (Ids 9 and 10, an experimental 64x128-tile screen and an fp4
 *                      screen of round 2, are retired: WLD_E_ARG.) */
#define WLD_OPT_PREFILTER 1
#define WLD_OPT_SCREEN 2
#define WLD_OPT_TILE_ORDER 3
#define WLD_OPT_ALL_PLANES 4
#define WLD_OPT_MFMA_LAYOUT 5
#define WLD_OPT_VALU_PLAIN 6
#define WLD_OPT_STAGING_ROWS 7
#define WLD_OPT_HOST_BATCH_PAIRS 8
#define WLD_OPT_REF_SUMS 11
#define WLD_OPT_FUSED_SCAN 12
#define WLD_OPT_SCREEN_FP6 13
#define WLD_OPT_TEST_GUARD 14
#define WLD_OPT_FP6_PAIRS_MIN_TILES 15
#define WLD_OPT_I8_PAIRS 16
int wld_set_option(wld_ctx *ctx, int option, int64_t value);
int wld_get_option(wld_ctx *ctx, int option, int64_t *value);

/* Rows of PairStore<LdStats> (lib.rs:523-576) as structure-of-arrays, in the
 * reference's order: 256x256 chunks in triu_index order (lib.rs:623-635:
 * chunk rows descending, columns ascending), then site_a, then site_b
 * ascending.  Site indices are PARENT indices (lib.rs:662-663).  Only rows
 * with r2 > r2_threshold (strict, lib.rs:660; NaN never passes). */
typedef struct {
    uint64_t n;
    uint32_t *site_a;
    uint32_t *site_b;
    float *d;
    float *d_prime;
    float *r2;
} wld_pairs;
void wld_pairs_free(wld_pairs *p); /* only for host results made by this library */

/* progress_report (lib.rs:582, main.rs:184-188).  Called on the calling
 * thread (never from a worker): once with 0 before any work (lib.rs:584, by
 * wld_all_weighted_ld_pairs), then once per completed 256x256 chunk with the
 * number of pairs in the chunks completed before it — the previous value of
 * lib.rs's fetch_add counter (lib.rs:670-674); values never decrease. */
typedef void (*wld_progress_fn)(uint64_t pairs_done, void *user);

/* Drop-in for all_weighted_ld_pairs (lib.rs:578-684).  Blocking.  sites is
 * SiteSet.buffer (n_sites*n_seqs bytes, host memory), site_map the SiteSet's
 * site_map (NULL = identity), weights n_seqs floats.  Allocates out's host
 * arrays (release with wld_pairs_free). */
int wld_all_weighted_ld_pairs(wld_ctx *ctx, const uint8_t *sites, size_t n_sites, size_t n_seqs,
                              const uint64_t *site_map, const float *weights, float r2_threshold,
                              wld_progress_fn progress, void *user, wld_pairs *out);

/* Drop-in for single_weighted_ld_pair (lib.rs:390-521) with the histograms of
 * a and b taken from the slices themselves (as SiteSet does).  Returns 1 and
 * fills out[3] = {d, d_prime, r2} for Some, 0 for None, <0 on error. */
int wld_single_weighted_ld_pair(wld_ctx *ctx, const uint8_t *a, const uint8_t *b,
                                const float *weights, size_t n_seqs, float out[3]);

/* ---- staged API: inputs resident in HBM, shardable, results on device ---- */

/* Uploads a SiteSet (host pointers) and encodes it on the device: per-site
 * histogram -> major/minor (lib.rs:126-140, hoisted out of the pair loop)
 * -> per-sequence codes and weight planes.  Replaces any previous load. */
int wld_load(wld_ctx *ctx, const uint8_t *sites, size_t n_sites, size_t n_seqs,
             const uint64_t *site_map, const float *weights);
/* Same, from device pointers already resident in HBM (d_sites: n_sites*n_seqs
 * bytes site-major; d_weights: n_seqs floats; site_map host, may be NULL). */
int wld_load_device(wld_ctx *ctx, const void *d_sites, size_t n_sites, size_t n_seqs,
                    const uint64_t *site_map, const void *d_weights);

/* Device pre-pass, replacing the host steps of
 * main.rs:139-156 for the staged API: from the UNFILTERED SiteSet buffer
 * (n_sites*n_seqs site-major Symbol codes, lib.rs:163), keeps the sites for
 * which is_site_of_interest(site, ceil(min_acgt*n_seqs), min_minor, max_minor)
 * holds (lib.rs:309-338; filter_by, lib.rs:230-251), computes Henikoff weights
 * on the kept sites (lib.rs:340-380) or unit weights if `unweighted`
 * (main.rs:150-153), and loads the kept set for wld_run with parent site
 * indices as its site_map.  Bit-identical to wld_siteset_filter_sites_of_interest
 * + wld_henikoff_weights + wld_load.  *n_kept receives the kept site count. */
int wld_load_filtered(wld_ctx *ctx, const uint8_t *sites, size_t n_sites, size_t n_seqs,
                      const uint64_t *site_map, float min_acgt, float min_minor, float max_minor,
                      int unweighted, size_t *n_kept);
/* Same, from a device pointer (read during the call only).  In both, site_map
 * is the unfiltered SiteSet's own map (host, NULL = identity); kept sites
 * report site_map[i] as their parent index, as filter_by composes it. */
int wld_load_filtered_device(wld_ctx *ctx, const void *d_sites, size_t n_sites, size_t n_seqs,
                             const uint64_t *site_map, float min_acgt, float min_minor, float max_minor,
                             int unweighted, size_t *n_kept);
/* After wld_load_filtered[_device]: the n_seqs weights (for the weights TSV,
 * main.rs:157-165) and the n_kept parent site indices. */
int wld_weights_copy(wld_ctx *ctx, float *out);
int wld_site_map_copy(wld_ctx *ctx, uint64_t *out);

/* Number of 256-site chunk rows n = ceil(n_sites/256) (lib.rs:615-619), and a
 * balanced contiguous partition of chunk rows [begin,end) for shard `shard` of
 * `n_shards` (equal pair counts up to chunk granularity).  Each shard's rows
 * are a contiguous run of the reference order; shards concatenate in
 * DESCENDING shard order (chunk rows descend in triu_index order). */
uint32_t wld_chunk_rows(size_t n_sites);
int wld_shard_chunk_rows(size_t n_sites, int n_shards, int shard, uint32_t *begin, uint32_t *end);

/* The reference's chunk sequence (lib.rs:615-634): n(n+1)/2 chunks of 256x256
 * sites, linear index i <-> (row, col) by triu_index, rows descending and
 * columns ascending; PairStore rows come chunk by chunk in this order.
 * wld_shard_chunks partitions it into contiguous linear ranges [begin,end) of
 * near-equal pair count (single-chunk granularity, finer than chunk rows);
 * shard 0 takes the LAST range, so shards concatenate in DESCENDING shard
 * order, as with wld_shard_chunk_rows.  wld_pairs_in_chunks counts the pairs
 * (a<b) of a range. */
uint32_t wld_chunks(size_t n_sites);
int wld_shard_chunks(size_t n_sites, int n_shards, int shard, uint32_t *begin, uint32_t *end);
uint64_t wld_pairs_in_chunks(size_t n_sites, uint32_t begin, uint32_t end);

/* Evaluates every pair (a<b) whose a lies in chunk rows [row_begin,row_end)
 * (pass 0, wld_chunk_rows() for all), filters r2 > r2_threshold and leaves
 * the rows on the device in reference order.  *n_rows receives the count. */
int wld_run(wld_ctx *ctx, float r2_threshold, uint32_t row_begin, uint32_t row_end,
            uint64_t *n_rows);
/* wld_run over the linear chunk range [chunk_begin,chunk_end) (end 0 = all):
 * the rows of those chunks, in reference order (all_weighted_ld_pairs'
 * par_iter over 0..n(n+1)/2, lib.rs:621-683, restricted to a sub-range). */
int wld_run_chunks(wld_ctx *ctx, float r2_threshold, uint32_t chunk_begin, uint32_t chunk_end,
                   uint64_t *n_rows);
/* The same run in two calls, for callers that overlap it with a collective:
 * wld_run_chunks_async enqueues the pair kernel and the row count on the
 * context's stream (wld_stream) and returns without waiting; when
 * d_count_out (device, 8 bytes) is given the run's row total lands there as a
 * uint64 on that stream.  wld_run_wait completes the run (host wait, staging
 * regrowth, reference-order assembly) exactly as wld_run_chunks would.  No
 * other call may touch the context in between. */
int wld_run_chunks_async(wld_ctx *ctx, float r2_threshold, uint32_t chunk_begin, uint32_t chunk_end,
                         void *d_count_out);
int wld_run_wait(wld_ctx *ctx, uint64_t *n_rows);
/* Orders ctx's next run after prev's enqueued one on the device, no host wait:
 * ctx's stream waits until prev's pair kernels (for a screened pass: its
 * screen kernel) have completed; prev's candidate launch, row count and
 * assembly may still overlap ctx's kernels.  For callers that pipeline runs
 * over several contexts (the N>1 step loop): one pair kernel at a time with
 * the next one already queued.  A no-op when prev has no run in flight;
 * WLD_E_STATE when ctx has one; WLD_E_ARG for device groups. */
int wld_run_after(wld_ctx *ctx, wld_ctx *prev);
/* The context's HIP stream (hipStream_t), for ordering caller work after a run. */
void *wld_stream(wld_ctx *ctx);
/* Runs the context's device work on the caller's HIP stream from now on
 * (a hipStream_t of the context's device; NULL: back to the context's own
 * stream).  Contexts given one stream run one after another in enqueue order
 * with nothing between their kernels (the N=1 pipelined loop: the next run
 * queued behind the previous one without a cross-queue event, cf.
 * wld_run_after, which then returns at once).  WLD_E_STATE during a run,
 * WLD_E_ARG for device groups.  The stream is borrowed: it must outlive its
 * use by ctx (set the context back to NULL, or destroy ctx, before destroying
 * the stream or the context that owns it); wld_destroy waits for the work ctx
 * queued on a borrowed stream. */
int wld_set_stream(wld_ctx *ctx, void *stream);
/* All pairs of the loaded set, any size, rows to host: runs the reference's
 * chunk sequence in batches of at most 2^31 pairs (one wld_run_chunks each),
 * appending each batch's rows to library-allocated host arrays in reference
 * order (release with wld_pairs_free); progress (may be NULL) is called per
 * completed chunk as in wld_progress_fn: the kernels count down each chunk's
 * tiles and log finished chunks to mapped host memory, which the calling
 * thread polls while the batch runs. */
int wld_run_host(wld_ctx *ctx, float r2_threshold, wld_progress_fn progress, void *user, wld_pairs *out);
/* Device pointers of the last run's rows (valid until the next run/load or
 * destroy; do not free). */
int wld_rows_device(wld_ctx *ctx, wld_pairs *view);
/* Copies the last run's rows to caller host arrays of at least n_rows each
 * (any pointer may be NULL to skip that column). */
int wld_rows_copy(wld_ctx *ctx, uint32_t *site_a, uint32_t *site_b, float *d, float *d_prime,
                  float *r2);
/* Device-to-device copy of the last run's rows into caller device buffers
 * (e.g. tensors handed to an RCCL gather); NULL skips a column.  Completes
 * before returning. */
int wld_rows_copy_device(wld_ctx *ctx, void *site_a, void *site_b, void *d, void *d_prime, void *r2);
/* Dense stats of every pair a<b of the loaded set into host n_sites*n_sites
 * row-major matrices (valid[a*L+b] = 1 for Some); for tests. */
int wld_dense(wld_ctx *ctx, float *d, float *d_prime, float *r2, uint8_t *valid);

typedef struct {
    int kernel;              /* WLD_KERNEL_VALU or WLD_KERNEL_MFMA actually used   */
    uint64_t pairs;          /* pairs evaluated (a<b) in the last run              */
    uint64_t rows;           /* rows that passed the threshold                     */
    double pair_kernel_ms;   /* HIP-event time of the pair phase (last run): the pair
                                kernel, or screen + candidate launch           */
    double order_ms;         /* HIP-event time of the ordering kernels (last run)  */
    double load_ms;          /* HIP-event time of the encode kernel (last load)    */
    uint64_t pair_kernel_launches; /* 2 when screened: screen + candidate tiles */
    int weight_shift;        /* fixed-point exponent of the MFMA weight planes     */
    int mfma_planes;         /* weight-digit planes the MFMA kernel multiplies (1-3; all-zero planes skipped) */
    uint64_t tiles;          /* 64x64 site tiles of the last run                   */
    uint64_t candidate_tiles;/* tiles computed with every plane (= tiles unless screened) */
    double screen_ms;        /* HIP-event time of the screen launch (0 if none)    */
    int screened;            /* 1: the last run ran the one-plane i8 screen; 3: the two-plane
                                i8 screen; 4: (lib.rs's order) an i8 pass (the top two digit
                                planes) staging the pairs its bound cannot reject, each then
                                summed alone in lib.rs's order; 0: none */
    int ref_sums;            /* 1: the last run summed in lib.rs's f32 order (WLD_OPT_REF_SUMS) */
    uint64_t candidate_blocks; /* 16x16 sub-blocks of the candidate tiles holding a pair the screen
                                  could not reject (16 x candidate_tiles unless screened); with
                                  WLD_OPT_REF_SUMS only these are computed */
    uint64_t candidate_pairs; /* screened == 4: the pairs summed one by one in lib.rs's order */
    int screen_fp6;          /* screened == 1 on fp6 x fp4 block-scaled MFMA (WLD_OPT_SCREEN_FP6), not i8;
                                2: the fp6 screen gave the pass up (more than a sixteenth of the tiles were
                                candidates) and it re-ran on the i8 screen */
    int fp6_sampled;         /* 1: this pass's screen (fp6 or i8) was chosen by the fp6 screen's sample run
                                (WLD_OPT_SCREEN_FP6 1: about 1/64 of the tiles screened first, at a
                                threshold not decided before) */
    uint64_t progress_filled; /* per-chunk progress (wld_run_host with a callback): chunk reports the
                                 host made up from the chunk pair counts because the pass's log lacked
                                 their entries once it had completed; 0 unless the kernels' chunk
                                 accounting lost a count (the tests assert 0) */
} wld_run_stats;
int wld_last_stats(wld_ctx *ctx, wld_run_stats *out);

#ifdef __cplusplus
}
#endif
#endif /* WEIGHTEDLD_H */
