/*
 * wld_oracle.c — CPU restatement of the WeightedLD Rust crate's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP path
 * and the "port" CPU baseline in bench.py.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product library
 * (weightedld_amd/libweightedld.so) never links or calls it.
 *
 * It restates rust/weighted_ld/src/lib.rs (reference @ /root/reference) in
 * plain C, with the `simd` feature semantics:
 *   - Symbol codes              lib.rs:20-64   (A,C,G,T,Missing,Unknown = 0..5)
 *   - SymbolHistogram           lib.rs:72-141  (major_minor_symbols :126-140)
 *   - read_fasta quirks         lib.rs:277-307 (each non-'>' line is a sequence,
 *                                               its '\n' becomes an Unknown site)
 *   - SiteSet::from_multiseq    lib.rs:176-206 (site-major buffer)
 *   - is_site_of_interest       lib.rs:309-338
 *   - henikoff_weights          lib.rs:340-380
 *   - single_weighted_ld_pair   lib.rs:390-521 (8-lane f32 accumulation :416-453,
 *                                               scalar tail :461-480, epilogue :482-520)
 *   - all_weighted_ld_pairs     lib.rs:578-684 (256x256 triangular chunks,
 *                                               triu_index order :623-632,
 *                                               strict r2 > threshold :660)
 *
 * Parity notes:
 *   - The Rust crate cannot be built in this image (no cargo/rustc; the simd
 *     feature needs nightly + packed_simd_2 0.3.5), so this restatement is
 *     pinned by the lib.rs unit-test known answers and by golden vectors from
 *     the Python reference (tests/golden/, made by oracle/gen_golden.py).
 *   - packed_simd's f32x8::sum() horizontal order is not pinned by any
 *     reference test.  packed_simd_2 0.3.5 (Cargo.lock:531-534)
 *     documents a tree reduction but implements sum() on x86 as
 *     simd_reduce_add_ordered(v, 0.0), i.e. ((((0+x0)+x1)+...)+x7) — the
 *     default here.  wldo_set_hsum_order(1) selects the documented tree
 *     ((x0+x1)+(x2+x3))+((x4+x5)+(x6+x7)) so tests can report how much the
 *     choice matters.
 *   - Compiled with -ffp-contract=off: Rust does not contract a*b+c.
 */
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { SYM_A = 0, SYM_C, SYM_G, SYM_T, SYM_MISSING, SYM_UNKNOWN };

typedef float f32x8 __attribute__((vector_size(32)));
typedef int32_t i32x8 __attribute__((vector_size(32)));

/* lib.rs:53-64 */
uint8_t wldo_symbol_from_char(uint32_t c) {
    switch (c) {
    case 'a': case 'A': return SYM_A;
    case 'c': case 'C': return SYM_C;
    case 'g': case 'G': return SYM_G;
    case 't': case 'T': return SYM_T;
    case '-': return SYM_MISSING;
    default: return SYM_UNKNOWN;
    }
}

/* lib.rs:98-104 */
void wldo_histogram(const uint8_t *site, size_t n, uint64_t hist[6]) {
    for (int s = 0; s < 6; ++s) hist[s] = 0;
    for (size_t i = 0; i < n; ++i) hist[site[i]] += 1;
}

/* lib.rs:126-140 — strict '>' so ties keep the earlier symbol of A,C,G,T,-;
 * Unknown is never eligible.  -1 stands for None. */
void wldo_major_minor(const uint64_t hist[6], int *major, int *minor) {
    int maj = -1, mnr = -1;
    for (int s = SYM_A; s <= SYM_MISSING; ++s) {
        uint64_t maj_c = maj >= 0 ? hist[maj] : 0;
        uint64_t min_c = mnr >= 0 ? hist[mnr] : 0;
        if (hist[s] > maj_c) {
            mnr = maj;
            maj = s;
        } else if (hist[s] > min_c) {
            mnr = s;
        }
    }
    *major = maj;
    *minor = mnr;
}

/* lib.rs:309-338 */
int wldo_is_site_of_interest(const uint8_t *site, size_t n, size_t min_acgt,
                             float min_minor, float max_minor) {
    uint64_t h[6];
    wldo_histogram(site, n, h);
    uint64_t acgt = h[0] + h[1] + h[2] + h[3];
    if (acgt <= min_acgt) return 0;
    int maj, mnr;
    wldo_major_minor(h, &maj, &mnr);
    if (maj < 0 || mnr < 0) return 0;
    float maj_count = (float)h[maj];
    float min_count = (float)h[mnr];
    float minor_frac = min_count / (min_count + maj_count);
    if (minor_frac < min_minor || minor_frac > max_minor) return 0;
    return 1;
}

/* main.rs:139: ceil(f32 min_acgt * n_seqs) as usize */
size_t wldo_min_acgt_count(float min_acgt, size_t n_seqs) {
    float v = ceilf(min_acgt * (float)n_seqs);
    return v <= 0.0f ? 0 : (size_t)v;
}

/* lib.rs:277-307 + lib.rs:176-206.  Reads FASTA the way the Rust crate does:
 * every line that does not start with '>' is one sequence, and read_line keeps
 * the trailing '\n' (and a '\r'), so each becomes an Unknown site.  Returns
 * 0 on success, -1 on I/O error, -2 where the Rust code would panic
 * ("Not all sequences have the same number of symbols", lib.rs:180-182, or
 * indexing sequences[0] of an empty file, lib.rs:178).
 * The buffer is site-major: buffer[site * n_seqs + seq].  Free with wldo_free. */
int wldo_read_fasta(const char *path, uint8_t **buffer, size_t *n_seqs, size_t *n_sites) {
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    char *data = (char *)malloc((size_t)sz + 1);
    if (!data) { fclose(f); return -1; }
    size_t got = fread(data, 1, (size_t)sz, f);
    fclose(f);
    data[got] = 0;

    /* pass 1: sequence lines and their lengths (in chars; input is ASCII) */
    size_t cap = 64, nseq = 0;
    size_t *start = (size_t *)malloc(cap * sizeof(size_t));
    size_t *len = (size_t *)malloc(cap * sizeof(size_t));
    size_t pos = 0;
    while (pos < got) {
        size_t e = pos;
        while (e < got && data[e] != '\n') ++e;
        size_t line_len = (e < got) ? e - pos + 1 : e - pos; /* keep '\n' */
        if (data[pos] != '>') {
            if (nseq == cap) {
                cap *= 2;
                start = (size_t *)realloc(start, cap * sizeof(size_t));
                len = (size_t *)realloc(len, cap * sizeof(size_t));
            }
            start[nseq] = pos;
            len[nseq] = line_len;
            ++nseq;
        }
        pos += line_len;
    }
    if (nseq == 0) { free(start); free(len); free(data); return -2; }
    size_t nsite = len[0];
    for (size_t i = 0; i < nseq; ++i)
        if (len[i] != nsite) { free(start); free(len); free(data); return -2; }
    uint8_t *buf = (uint8_t *)malloc((nseq * nsite) > 0 ? nseq * nsite : 1);
    for (size_t s = 0; s < nseq; ++s)
        for (size_t j = 0; j < nsite; ++j)
            buf[j * nseq + s] = wldo_symbol_from_char((unsigned char)data[start[s] + j]);
    free(start); free(len); free(data);
    *buffer = buf;
    *n_seqs = nseq;
    *n_sites = nsite;
    return 0;
}

void wldo_free(void *p) { free(p); }

/* lib.rs:360-380 */
static void henikoff_site_contributions(const uint8_t *site, size_t n, float *contrib) {
    uint64_t h[6];
    wldo_histogram(site, n, h);
    size_t distinct = 0;
    for (int s = 0; s <= SYM_MISSING; ++s) distinct += h[s] > 0;
    float distinct_f = (float)distinct;
    float total = 0.0f;
    for (size_t i = 0; i < n; ++i) {
        if (site[i] <= SYM_MISSING) {
            contrib[i] = 1.0f / (distinct_f * (float)h[site[i]]);
            total += contrib[i];
        }
    }
    float mean = total / distinct_f;
    for (size_t i = 0; i < n; ++i)
        if (site[i] > SYM_MISSING) contrib[i] = mean;
}

/* lib.rs:340-358.  sum_axis(Axis(0)) over a (n_sites, n_seqs) C-order array
 * adds the site rows in order (ndarray's non-contiguous-axis path); the
 * max fold starts at 0.0 and uses f32::max. */
void wldo_henikoff_weights(const uint8_t *buf, size_t n_sites, size_t n_seqs, float *out) {
    float *contrib = (float *)calloc(n_seqs ? n_seqs : 1, sizeof(float));
    for (size_t i = 0; i < n_seqs; ++i) out[i] = 0.0f;
    for (size_t s = 0; s < n_sites; ++s) {
        for (size_t i = 0; i < n_seqs; ++i) contrib[i] = 0.0f;
        henikoff_site_contributions(buf + s * n_seqs, n_seqs, contrib);
        for (size_t i = 0; i < n_seqs; ++i) out[i] = out[i] + contrib[i];
    }
    float mx = 0.0f;
    for (size_t i = 0; i < n_seqs; ++i) mx = fmaxf(mx, out[i]);
    for (size_t i = 0; i < n_seqs; ++i) out[i] = out[i] / mx;
    free(contrib);
}

/* Horizontal f32x8 sum (lib.rs:447-452): 0 = ordered from 0.0 (default), 1 = tree. */
static int g_hsum_tree = 0;
void wldo_set_hsum_order(int tree) { g_hsum_tree = tree != 0; }
int wldo_get_hsum_order(void) { return g_hsum_tree; }

static float hsum8(f32x8 v) {
    if (g_hsum_tree) return ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
    float s = 0.0f;
    for (int j = 0; j < 8; ++j) s += v[j];
    return s;
}

/* lib.rs:390-521.  Returns 1 (Some) and fills out[0..3] = {d, d_prime, r2},
 * or 0 (None) when either site lacks a major or a minor symbol. */
int wldo_single_pair_mm(const uint8_t *a, int a_maj, int a_min, const uint8_t *b, int b_maj,
                        int b_min, const float *w, size_t n, float out[3]) {
    if (a_maj < 0 || a_min < 0 || b_maj < 0 || b_min < 0) return 0;
    const uint8_t am = (uint8_t)a_maj, an = (uint8_t)a_min;
    const uint8_t bm = (uint8_t)b_maj, bn = (uint8_t)b_min;
    size_t simd_end = (n / 8) * 8;

    /* :416-445 — 8 lanes, op for op like packed_simd's u8x8 eq / f32x8 select
     * (GCC vector types; with -march=x86-64-v3 this is AVX2 like the reference's
     * RUSTFLAGS=-C target-cpu=native build, README.md:88-97). */
    f32x8 tw = {0}, pa = {0}, pb = {0}, l3 = {0};
    for (size_t seq = 0; seq < simd_end; seq += 8) {
        i32x8 av, bv;
        for (int j = 0; j < 8; ++j) {
            av[j] = a[seq + j];
            bv[j] = b[seq + j];
        }
        const i32x8 a_maj = av == (i32x8){am, am, am, am, am, am, am, am};
        const i32x8 a_min = av == (i32x8){an, an, an, an, an, an, an, an};
        const i32x8 b_maj = bv == (i32x8){bm, bm, bm, bm, bm, bm, bm, bm};
        const i32x8 b_min = bv == (i32x8){bn, bn, bn, bn, bn, bn, bn, bn};
        const i32x8 mask = (a_maj | a_min) & (b_maj | b_min);
        f32x8 wv;
        memcpy(&wv, w + seq, sizeof wv);
        const i32x8 wbits = (i32x8)wv & mask; /* mask.select(weight, zero) */
        tw += (f32x8)wbits;
        pa += (f32x8)(wbits & a_maj);
        pb += (f32x8)(wbits & b_maj);
        l3 += (f32x8)(wbits & (a_maj & b_maj));
    }
    /* :447-452 — horizontal sums (see header) */
    float total_weight = hsum8(tw), PA = hsum8(pa), PB = hsum8(pb), ld3 = hsum8(l3);
    /* :461-480 — scalar tail */
    for (size_t seq = simd_end; seq < n; ++seq) {
        if (!(a[seq] == am || a[seq] == an)) continue;
        if (!(b[seq] == bm || b[seq] == bn)) continue;
        total_weight += w[seq];
        if (a[seq] == am) PA += w[seq];
        if (b[seq] == bm) PB += w[seq];
        if (a[seq] == am && b[seq] == bm) ld3 += w[seq];
    }
    /* :482-520 */
    float ld_obs[4];
    float Pa = total_weight - PA;
    float Pb = total_weight - PB;
    ld_obs[3] = ld3;
    ld_obs[2] = PA - ld_obs[3];
    ld_obs[1] = PB - ld_obs[3];
    ld_obs[0] = Pa - ld_obs[1];
    PA /= total_weight;
    PB /= total_weight;
    Pa /= total_weight;
    Pb /= total_weight;
    ld_obs[0] /= total_weight;
    ld_obs[1] /= total_weight;
    ld_obs[2] /= total_weight;
    ld_obs[3] /= total_weight;
    float PAB = PA * PB, PAb = PA * Pb, PaB = Pa * PB, Pab = Pa * Pb;
    float d = ((PAB - ld_obs[3]) + (Pab - ld_obs[0]) + (ld_obs[2] - PAb) + (ld_obs[1] - PaB)) / 4.0f;
    float den;
    if (d < 0.0f) {
        den = fmaxf(-ld_obs[0], -ld_obs[3]);
        if (den == 0.0f) den = fminf(-ld_obs[0], -ld_obs[3]);
    } else {
        den = fminf(ld_obs[1], ld_obs[2]);
        if (den == 0.0f) den = fmaxf(ld_obs[1], ld_obs[2]);
    }
    float d_prime = d / den;
    float r2 = d * d / (PA * Pa * PB * Pb);
    out[0] = d;
    out[1] = d_prime;
    out[2] = r2;
    return 1;
}

int wldo_single_pair(const uint8_t *a, const uint8_t *b, const float *w, size_t n, float out[3]) {
    uint64_t ha[6], hb[6];
    int am, an, bm, bn;
    wldo_histogram(a, n, ha);
    wldo_histogram(b, n, hb);
    wldo_major_minor(ha, &am, &an);
    wldo_major_minor(hb, &bm, &bn);
    return wldo_single_pair_mm(a, am, an, b, bm, bn, w, n, out);
}

/* lib.rs:623-632, f32 arithmetic as in the reference */
void wldo_triu_index(size_t n, size_t i, size_t *row, size_t *col) {
    float root = (sqrtf((float)i * 8.0f + 1.0f) - 1.0f) / 2.0f;
    size_t rf = (size_t)floorf(root);
    *row = n - rf - 1;
    *col = *row + i - (rf * (rf + 1) / 2);
}

/* ---------------- all_weighted_ld_pairs (lib.rs:578-684) ---------------- */

typedef struct {
    uint64_t n;
    uint64_t *site_a, *site_b;
    float *d, *d_prime, *r2;
} wldo_rows;

typedef struct {
    size_t n, cap;
    uint64_t *a, *b;
    float *v; /* d, d', r2 interleaved */
} chunk_rows;

typedef struct {
    const uint8_t *buf;
    size_t n_sites, n_seqs;
    const uint64_t *site_map;
    const float *w;
    float thr;
    const int8_t *maj, *mnr;
    size_t n, chunk_count, chunk_size;
    size_t chunk_lo, chunk_hi; /* linear chunk range to process */
    atomic_size_t next;
    atomic_ullong pairs_done;
    chunk_rows *out;
} job_t;

static void push_row(chunk_rows *c, uint64_t a, uint64_t b, const float v[3]) {
    if (c->n == c->cap) {
        c->cap = c->cap ? c->cap * 2 : 1024;
        c->a = (uint64_t *)realloc(c->a, c->cap * sizeof(uint64_t));
        c->b = (uint64_t *)realloc(c->b, c->cap * sizeof(uint64_t));
        c->v = (float *)realloc(c->v, c->cap * 3 * sizeof(float));
    }
    c->a[c->n] = a;
    c->b[c->n] = b;
    memcpy(c->v + 3 * c->n, v, 3 * sizeof(float));
    c->n++;
}

static void *worker(void *arg) {
    job_t *J = (job_t *)arg;
    for (;;) {
        size_t i = atomic_fetch_add(&J->next, 1);
        if (i >= J->chunk_hi) break;
        size_t ca, cb;
        wldo_triu_index(J->n, i, &ca, &cb);
        size_t a0 = ca * J->chunk_size, a1 = a0 + J->chunk_size;
        size_t b0 = cb * J->chunk_size, b1 = b0 + J->chunk_size;
        if (a1 > J->n_sites) a1 = J->n_sites;
        if (b1 > J->n_sites) b1 = J->n_sites;
        chunk_rows *c = &J->out[i - J->chunk_lo];
        uint64_t computed = 0;
        for (size_t a = a0; a < a1; ++a) {
            for (size_t b = b0; b < b1; ++b) {
                if (b <= a) continue;
                ++computed;
                float v[3];
                if (wldo_single_pair_mm(J->buf + a * J->n_seqs, J->maj[a], J->mnr[a],
                                        J->buf + b * J->n_seqs, J->maj[b], J->mnr[b], J->w,
                                        J->n_seqs, v)) {
                    if (v[2] > J->thr) {
                        uint64_t pa = J->site_map ? J->site_map[a] : a;
                        uint64_t pb = J->site_map ? J->site_map[b] : b;
                        push_row(c, pa, pb, v);
                    }
                }
            }
        }
        atomic_fetch_add(&J->pairs_done, computed);
    }
    return NULL;
}

/* Computes chunks [chunk_lo, chunk_hi) of the triu chunk sequence (the full
 * sequence is [0, n(n+1)/2)), threaded over n_threads with dynamic chunk
 * claiming like rayon's work stealing, and concatenates per-chunk rows in
 * chunk order (rayon's order-preserving collect, lib.rs:678-679).
 * Returns the number of pairs evaluated (a<b), or -1 on bad arguments. */
int64_t wldo_all_pairs_range(const uint8_t *buf, size_t n_sites, size_t n_seqs,
                             const uint64_t *site_map, const float *w, float thr, int n_threads,
                             size_t chunk_lo, size_t chunk_hi, wldo_rows *out) {
    const size_t chunk_size = 256;
    size_t n = n_sites / chunk_size + ((n_sites % chunk_size) > 0);
    size_t chunk_count = n * (n + 1) / 2;
    if (chunk_hi > chunk_count) chunk_hi = chunk_count;
    if (chunk_lo > chunk_hi) return -1;
    if (n_threads < 1) n_threads = 1;

    int8_t *maj = (int8_t *)malloc(n_sites ? n_sites : 1);
    int8_t *mnr = (int8_t *)malloc(n_sites ? n_sites : 1);
    for (size_t s = 0; s < n_sites; ++s) {
        uint64_t h[6];
        int mj, mn;
        wldo_histogram(buf + s * n_seqs, n_seqs, h);
        wldo_major_minor(h, &mj, &mn);
        maj[s] = (int8_t)mj;
        mnr[s] = (int8_t)mn;
    }
    job_t J;
    memset(&J, 0, sizeof(J));
    J.buf = buf; J.n_sites = n_sites; J.n_seqs = n_seqs; J.site_map = site_map; J.w = w;
    J.thr = thr; J.maj = maj; J.mnr = mnr; J.n = n; J.chunk_count = chunk_count;
    J.chunk_size = chunk_size; J.chunk_lo = chunk_lo; J.chunk_hi = chunk_hi;
    atomic_init(&J.next, chunk_lo);
    atomic_init(&J.pairs_done, 0);
    size_t nch = chunk_hi - chunk_lo;
    J.out = (chunk_rows *)calloc(nch ? nch : 1, sizeof(chunk_rows));

    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)n_threads);
    for (int t = 0; t < n_threads; ++t) pthread_create(&th[t], NULL, worker, &J);
    for (int t = 0; t < n_threads; ++t) pthread_join(th[t], NULL);
    free(th);

    uint64_t total = 0;
    for (size_t c = 0; c < nch; ++c) total += J.out[c].n;
    out->n = total;
    size_t alloc = total ? total : 1;
    out->site_a = (uint64_t *)malloc(alloc * sizeof(uint64_t));
    out->site_b = (uint64_t *)malloc(alloc * sizeof(uint64_t));
    out->d = (float *)malloc(alloc * sizeof(float));
    out->d_prime = (float *)malloc(alloc * sizeof(float));
    out->r2 = (float *)malloc(alloc * sizeof(float));
    uint64_t k = 0;
    for (size_t c = 0; c < nch; ++c) {
        chunk_rows *cr = &J.out[c];
        for (size_t r = 0; r < cr->n; ++r, ++k) {
            out->site_a[k] = cr->a[r];
            out->site_b[k] = cr->b[r];
            out->d[k] = cr->v[3 * r];
            out->d_prime[k] = cr->v[3 * r + 1];
            out->r2[k] = cr->v[3 * r + 2];
        }
        free(cr->a); free(cr->b); free(cr->v);
    }
    free(J.out);
    free(maj);
    free(mnr);
    return (int64_t)atomic_load(&J.pairs_done);
}

int64_t wldo_all_pairs(const uint8_t *buf, size_t n_sites, size_t n_seqs, const uint64_t *site_map,
                       const float *w, float thr, int n_threads, wldo_rows *out) {
    return wldo_all_pairs_range(buf, n_sites, n_seqs, site_map, w, thr, n_threads, 0, (size_t)-1,
                                out);
}

void wldo_rows_free(wldo_rows *r) {
    free(r->site_a); free(r->site_b); free(r->d); free(r->d_prime); free(r->r2);
    memset(r, 0, sizeof(*r));
}

/* f64 "truth" for diagnostics: the same masked sums accumulated in double and
 * the lib.rs:482-520 epilogue evaluated in double (what the f32 results
 * approximate).  Used by the tests to tell a GPU result that is closer to the
 * exact value than the f32 reference from a wrong one. */
int wldo_single_pair_f64(const uint8_t *a, int am, int an, const uint8_t *b, int bm, int bn, const float *w,
                         size_t n, double out[3]) {
    if (am < 0 || an < 0 || bm < 0 || bn < 0) return 0;
    double T = 0, PA = 0, PB = 0, l3 = 0;
    for (size_t k = 0; k < n; ++k) {
        int ain = a[k] == am || a[k] == an, bin = b[k] == bm || b[k] == bn;
        if (!(ain && bin)) continue;
        T += w[k];
        if (a[k] == am) PA += w[k];
        if (b[k] == bm) PB += w[k];
        if (a[k] == am && b[k] == bm) l3 += w[k];
    }
    double o3 = l3, o2 = PA - o3, o1 = PB - o3, Pa = T - PA, Pb = T - PB, o0 = Pa - o1;
    PA /= T; PB /= T; Pa /= T; Pb /= T; o0 /= T; o1 /= T; o2 /= T; o3 /= T;
    double d = ((PA * PB - o3) + (Pa * Pb - o0) + (o2 - PA * Pb) + (o1 - Pa * PB)) / 4.0;
    double den;
    if (d < 0) {
        den = fmax(-o0, -o3);
        if (den == 0) den = fmin(-o0, -o3);
    } else {
        den = fmin(o1, o2);
        if (den == 0) den = fmax(o1, o2);
    }
    out[0] = d;
    out[1] = d / den;
    out[2] = d * d / (PA * Pa * PB * Pb);
    return 1;
}

void wldo_all_pairs_dense_f64(const uint8_t *buf, size_t n_sites, size_t n_seqs, const float *w, double *d,
                              double *dp, double *r2, uint8_t *valid) {
    int *mm = (int *)malloc(2 * (n_sites ? n_sites : 1) * sizeof(int));
    for (size_t s = 0; s < n_sites; ++s) {
        uint64_t h[6];
        wldo_histogram(buf + s * n_seqs, n_seqs, h);
        wldo_major_minor(h, &mm[2 * s], &mm[2 * s + 1]);
    }
    for (size_t a = 0; a < n_sites; ++a)
        for (size_t b = a + 1; b < n_sites; ++b) {
            double v[3] = {0, 0, 0};
            size_t k = a * n_sites + b;
            valid[k] = (uint8_t)wldo_single_pair_f64(buf + a * n_seqs, mm[2 * a], mm[2 * a + 1], buf + b * n_seqs,
                                                     mm[2 * b], mm[2 * b + 1], w, n_seqs, v);
            d[k] = v[0];
            dp[k] = v[1];
            r2[k] = v[2];
        }
    free(mm);
}

/* Dense variant for tests: stats for every a<b written to row-major
 * n_sites x n_sites matrices; valid[a*L+b] = 1 for Some, 0 for None. */
void wldo_all_pairs_dense(const uint8_t *buf, size_t n_sites, size_t n_seqs, const float *w,
                          float *d, float *dp, float *r2, uint8_t *valid) {
    for (size_t a = 0; a < n_sites; ++a) {
        uint64_t ha[6];
        int am, an;
        wldo_histogram(buf + a * n_seqs, n_seqs, ha);
        wldo_major_minor(ha, &am, &an);
        for (size_t b = a + 1; b < n_sites; ++b) {
            uint64_t hb[6];
            int bm, bn;
            wldo_histogram(buf + b * n_seqs, n_seqs, hb);
            wldo_major_minor(hb, &bm, &bn);
            float v[3] = {0, 0, 0};
            int ok = wldo_single_pair_mm(buf + a * n_seqs, am, an, buf + b * n_seqs, bm, bn, w,
                                         n_seqs, v);
            size_t k = a * n_sites + b;
            valid[k] = (uint8_t)ok;
            d[k] = v[0];
            dp[k] = v[1];
            r2[k] = v[2];
        }
    }
}
